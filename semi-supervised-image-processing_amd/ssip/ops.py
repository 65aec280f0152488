"""Tensor-level wrappers over the C ABI (include/ssip.h).

Each function takes torch tensors that already live on the HIP device,
checks shapes/dtypes on the host, and launches on the current torch stream.
No function here falls back to a torch op.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import ctypes
import os

import torch

from . import _lib
from ._lib import ConvDesc, call

_DT = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16}


def dtype_code(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"ssip: unsupported activation dtype {t.dtype}") from None


def _p(t: Optional[torch.Tensor]):
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("ssip: tensor must be on the HIP device")
    if not t.is_contiguous():
        raise ValueError("ssip: tensor must be contiguous")
    return _lib.ptr(t)


def stream_ptr() -> int:
    """Raw hipStream_t of the calling thread's current stream (the plain
    torch.cuda.current_stream() path costs ~8 us per call; a step makes ~130)."""
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def wait_stream(dst: "torch.cuda.Stream", src: "torch.cuda.Stream") -> None:
    """dst waits for the work enqueued on src so far (torch's wait_stream);
    recorded into an active launch plan as an event record / wait pair."""
    dst.wait_stream(src)
    r = _lib.RECORDER
    if r is not None:
        r.wait_stream(dst.cuda_stream, src.cuda_stream)


def host_callback(fn, *args):
    """Run host work that issues device work outside the C ABI (collectives).
    Inside a launch-plan recording this ends a plan segment and is re-run at
    that point of every replay (its own launches are not recorded)."""
    r = _lib.RECORDER
    if r is None:
        return fn(*args)
    r.callback(fn, args)
    _lib.RECORDER = None
    try:
        return fn(*args)
    finally:
        _lib.RECORDER = r


def counters_add(counters, delta: int = 1) -> None:
    """tensor += delta for a list of int64 one-element device tensors, one launch."""
    for i in range(0, len(counters), 64):
        chunk = counters[i:i + 64]
        arr = (ctypes.c_void_p * len(chunk))(*[_p(t) for t in chunk])
        call("ssip_counters_add", len(chunk), arr, int(delta), stream_ptr())


# ---------------------------------------------------------------------------
# optional per-launch timing of the conv kernels (bench.py's roofline leg):
# HIP events recorded on the stream the kernels are launched on.
# ---------------------------------------------------------------------------
class ConvTimer:
    """HIP-event brackets around conv launches (bench.py's roofline leg).  Each
    record keeps the launch's algorithmic FLOPs and its algorithmic bytes (every
    operand tensor read once, every output written once), so a per-launch
    speed-of-light time max(FLOPs / MFMA peak, bytes / HBM peak) can be formed."""

    def __init__(self):
        self.records = []  # (kind, flops, bytes, start_event, end_event)

    def wrap(self, kind: str, flops: int, fn, *args, nbytes: int = 0):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn(*args)
        e.record()
        self.records.append((kind, flops, nbytes, s, e))

    def summary(self):
        """kind -> [flops, ms, launches, bytes]"""
        torch.cuda.synchronize()
        out = {}
        for kind, flops, nb, s, e in self.records:
            ms = s.elapsed_time(e)
            d = out.setdefault(kind, [0, 0.0, 0, 0])
            d[0] += flops
            d[1] += ms
            d[2] += 1
            d[3] += nb
        return out

    def sol(self, peak_flops: float, peak_bytes: float):
        """(sum over launches of max(flops / peak_flops, bytes / peak_bytes), measured sum), seconds"""
        torch.cuda.synchronize()
        sol = meas = 0.0
        for _, flops, nb, s, e in self.records:
            sol += max(flops / peak_flops, nb / peak_bytes)
            meas += s.elapsed_time(e) * 1e-3
        return sol, meas


def _nbytes(*ts) -> int:
    """Bytes of the distinct tensors given (None skipped, aliases counted once)."""
    seen, n = set(), 0
    for t in ts:
        if t is None or t.data_ptr() in seen:
            continue
        seen.add(t.data_ptr())
        n += t.numel() * t.element_size()
    return n


_timer = None


def set_conv_timer(t):
    global _timer
    _timer = t


# ---------------------------------------------------------------------------
# convolution
# ---------------------------------------------------------------------------
_desc_cache = {}  # ConvGeom -> its C descriptor (passed by reference, never written by the library)


@dataclass(frozen=True)
class ConvGeom:
    N: int
    H: int
    W: int
    C: int  # stored input channels (4 for the padded stem)
    K: int
    R: int
    S: int  # stored filter columns (8 for the padded stem)
    stride: int
    pad: int
    c_real: int
    s_real: int

    @property
    def P(self) -> int:
        return (self.H + 2 * self.pad - self.R) // self.stride + 1

    @property
    def Q(self) -> int:
        return (self.W + 2 * self.pad - self.s_real) // self.stride + 1

    def desc(self) -> ConvDesc:
        # the padded stem column (s = 7) must not change the output width:
        # Q is computed with the real filter width; the kernel only needs P/Q.
        d = _desc_cache.get(self)
        if d is None:
            d = _desc_cache[self] = ConvDesc(self.N, self.H, self.W, self.C, self.K, self.R, self.S, self.stride,
                                             self.pad, self.P, self.Q)
        return d

    def flops(self) -> int:
        return 2 * self.N * self.P * self.Q * self.K * self.c_real * self.R * self.s_real


# plans depend only on the geometry (and on SSIP_* tuning variables, read at
# each call by the library): memoised per (geometry, environment) for the host path
_plan_cache = {}


def _plan_env():
    return tuple(os.environ.get(k) for k in ("SSIP_HALO", "SSIP_CONV_FORCE", "SSIP_WGRAD_BIG"))


def conv_fwd_partial_floats(g: ConvGeom) -> int:
    key = ("pf", g, _plan_env())
    v = _plan_cache.get(key)
    if v is None:
        v = _plan_cache[key] = int(_lib.lib().ssip_conv_fwd_partial_floats(g.desc()))
    return v


def conv_fwd_partial_tiles(g: ConvGeom, dtype: torch.dtype) -> int:
    key = ("pt", g, dtype, _plan_env())
    t = _plan_cache.get(key)
    if t is None:
        t = int(_lib.lib().ssip_conv_fwd_partial_tiles(g.desc(), _DT[dtype]))
        if t <= 0:
            raise RuntimeError(_lib.lib().ssip_last_error().decode())
        _plan_cache[key] = t
    return t


def conv_fwd(g: ConvGeom, x: torch.Tensor, w_krsc: torch.Tensor, y: torch.Tensor,
             partial: Optional[torch.Tensor] = None) -> None:
    assert x.numel() == g.N * g.H * g.W * g.C, "conv_fwd: x shape"
    assert w_krsc.numel() == g.K * g.R * g.S * g.C, "conv_fwd: w shape"
    assert y.numel() == g.N * g.P * g.Q * g.K, "conv_fwd: y shape"
    assert x.dtype == w_krsc.dtype == y.dtype
    if partial is not None:
        assert partial.dtype == torch.float32 and partial.numel() >= conv_fwd_partial_floats(g)
    d = g.desc()
    if _timer is not None:
        _timer.wrap("fwd", g.flops(), call, "ssip_conv_fwd", d, dtype_code(x), _p(x), _p(w_krsc), _p(y), _p(partial),
                    stream_ptr(), nbytes=_nbytes(x, w_krsc, y))
        return
    call("ssip_conv_fwd", d, dtype_code(x), _p(x), _p(w_krsc), _p(y), _p(partial), stream_ptr())


def conv_fwd_ds_partial_tiles(g: ConvGeom, gds: ConvGeom, dtype: torch.dtype) -> int:
    """BN records per channel the fused forward writes for the downsample."""
    key = ("pds", g, gds, dtype, _plan_env(), os.environ.get("SSIP_NO_FWD_DSFUSE"))
    t = _plan_cache.get(key)
    if t is None:
        t = int(_lib.lib().ssip_conv_fwd_ds_partial_tiles(g.desc(), gds.desc(), _DT[dtype]))
        if t <= 0:
            raise RuntimeError(_lib.lib().ssip_last_error().decode())
        _plan_cache[key] = t
    return t


def conv_fwd_ds(g: ConvGeom, x: torch.Tensor, w_krsc: torch.Tensor, y: torch.Tensor, partial: Optional[torch.Tensor],
                gds: ConvGeom, wds: torch.Tensor, y_ds: torch.Tensor, partial_ds: Optional[torch.Tensor]) -> None:
    """A downsampling block's conv1 (3x3) and 1x1 downsample forwards over the
    same x in one launch (ssip_conv_fwd_ds)."""
    assert x.numel() == g.N * g.H * g.W * g.C and w_krsc.numel() == g.K * g.R * g.S * g.C, "conv_fwd_ds: shapes"
    assert y.numel() == y_ds.numel() == g.N * g.P * g.Q * g.K and wds.numel() == g.K * g.C, "conv_fwd_ds: shapes"
    assert x.dtype == w_krsc.dtype == y.dtype == wds.dtype == y_ds.dtype
    if partial is not None:
        assert partial.numel() >= conv_fwd_partial_floats(g) and partial_ds.numel() >= conv_fwd_partial_floats(gds)
    args = ("ssip_conv_fwd_ds", g.desc(), gds.desc(), dtype_code(x), _p(x), _p(w_krsc), _p(y), _p(partial),
            _p(wds), _p(y_ds), _p(partial_ds), stream_ptr())
    if _timer is not None:
        _timer.wrap("fwd", g.flops() + gds.flops(), call, *args, nbytes=_nbytes(x, w_krsc, y, wds, y_ds))
        return
    call(*args)


def conv_fwd_bias(g: ConvGeom, x: torch.Tensor, w_krsc: torch.Tensor, bias: torch.Tensor,
                  residual: Optional[torch.Tensor], relu: bool, y: torch.Tensor) -> None:
    """y = act(conv(x, w) + bias (+ residual)): eval-mode conv with its BN folded in (ssip_conv_fwd_bias)."""
    assert x.numel() == g.N * g.H * g.W * g.C, "conv_fwd_bias: x shape"
    assert w_krsc.numel() == g.K * g.R * g.S * g.C, "conv_fwd_bias: w shape"
    assert y.numel() == g.N * g.P * g.Q * g.K and bias.numel() == g.K, "conv_fwd_bias: y / bias shape"
    if residual is not None:
        assert residual.numel() == y.numel() and residual.dtype == y.dtype
    call("ssip_conv_fwd_bias", g.desc(), dtype_code(x), _p(x), _p(w_krsc), _p(bias), _p(residual), int(relu), _p(y),
         stream_ptr())


def conv_dgrad(g: ConvGeom, dy: torch.Tensor, w_crsk: torch.Tensor, dx: torch.Tensor,
               dx_add: Optional[torch.Tensor] = None) -> None:
    assert dy.numel() == g.N * g.P * g.Q * g.K, "conv_dgrad: dy shape"
    assert w_crsk.numel() == g.K * g.R * g.S * g.C, "conv_dgrad: w shape"
    assert dx.numel() == g.N * g.H * g.W * g.C, "conv_dgrad: dx shape"
    if dx_add is not None:
        assert dx_add.numel() == dx.numel() and dx_add.dtype == dx.dtype
    args = ("ssip_conv_dgrad", g.desc(), dtype_code(dy), _p(dy), _p(w_crsk), _p(dx), _p(dx_add), stream_ptr())
    if _timer is not None:
        # an in-place residual add (dx_add is dx) reads dx once more
        extra = dx.numel() * dx.element_size() if dx_add is not None and dx_add.data_ptr() == dx.data_ptr() else 0
        _timer.wrap("dgrad", g.flops(), call, *args, nbytes=_nbytes(dy, w_crsk, dx, dx_add) + extra)
        return
    call(*args)


def conv_dgrad_ds(g: ConvGeom, dy: torch.Tensor, w_crsk: torch.Tensor, gds: ConvGeom, dy_ds: torch.Tensor,
                  wds_crsk: torch.Tensor, dx: torch.Tensor) -> None:
    """dx = dgrad(conv g, dy) + dgrad(1x1/stride downsample gds, dy_ds) (ssip_conv_dgrad_ds)."""
    assert gds.R == 1 and gds.S == 1 and gds.pad == 0 and gds.stride == g.stride and (gds.P, gds.Q) == (g.P, g.Q)
    assert (gds.N, gds.H, gds.W, gds.C, gds.K) == (g.N, g.H, g.W, g.C, g.K), "conv_dgrad_ds: geometries differ"
    assert dy.numel() == dy_ds.numel() == g.N * g.P * g.Q * g.K, "conv_dgrad_ds: dy shape"
    assert w_crsk.numel() == g.K * g.R * g.S * g.C and wds_crsk.numel() == g.K * g.C, "conv_dgrad_ds: w shape"
    assert dx.numel() == g.N * g.H * g.W * g.C, "conv_dgrad_ds: dx shape"
    args = ("ssip_conv_dgrad_ds", g.desc(), dtype_code(dy), _p(dy), _p(w_crsk), _p(dy_ds), _p(wds_crsk), _p(dx),
            stream_ptr())
    if _timer is not None:
        _timer.wrap("dgrad", g.flops() + gds.flops(), call, *args, nbytes=_nbytes(dy, w_crsk, dy_ds, wds_crsk, dx))
        return
    call(*args)


def conv_dgrad_bn_partial_floats(g: ConvGeom) -> int:
    return int(_lib.lib().ssip_conv_dgrad_bn_partial_floats(g.desc()))


def conv_dgrad_bn_partial_tiles(g: ConvGeom, dtype: torch.dtype) -> int:
    t = int(_lib.lib().ssip_conv_dgrad_bn_partial_tiles(g.desc(), _DT[dtype]))
    if t <= 0:
        raise RuntimeError(_lib.lib().ssip_last_error().decode())
    return t


def conv_dgrad_bn(g: ConvGeom, dy: torch.Tensor, w_crsk: torch.Tensor, dx_add: Optional[torch.Tensor],
                  zmask: Optional[torch.Tensor], y: torch.Tensor, mean: torch.Tensor, invstd: torch.Tensor,
                  dpre: torch.Tensor, partial: torch.Tensor, mask_bits: Optional[torch.Tensor] = None,
                  mscale: Optional[torch.Tensor] = None, mshift: Optional[torch.Tensor] = None) -> None:
    """dpre = (dgrad(dy) + dx_add) * relu_mask plus the BN-backward partial
    sums ([C][tiles][2]) of the BN+ReLU below; the mask from zmask > 0, the
    forward's mask bits, or fma(y, mscale, mshift) > 0 (see include/ssip.h)."""
    assert dy.numel() == g.N * g.P * g.Q * g.K, "conv_dgrad_bn: dy shape"
    assert w_crsk.numel() == g.K * g.R * g.S * g.C, "conv_dgrad_bn: w shape"
    n = g.N * g.H * g.W * g.C
    assert dpre.numel() == n and y.numel() == n, "conv_dgrad_bn: activation shapes"
    assert zmask is None or zmask.numel() == n, "conv_dgrad_bn: zmask shape"
    assert mask_bits is None or (mask_bits.dtype == torch.uint8 and mask_bits.numel() * 8 == n)
    assert zmask is not None or mask_bits is not None or (mscale is not None and mshift is not None), \
        "conv_dgrad_bn: a ReLU-mask source is required"
    assert mean.numel() >= g.C and invstd.numel() >= g.C and mean.dtype == invstd.dtype == torch.float32
    assert partial.dtype == torch.float32 and partial.numel() >= conv_dgrad_bn_partial_floats(g)
    if dx_add is not None:
        assert dx_add.numel() == n and dx_add.dtype == dpre.dtype
    args = ("ssip_conv_dgrad_bn", g.desc(), dtype_code(dy), _p(dy), _p(w_crsk), _p(dx_add), _p(zmask),
            _p(mask_bits), _p(mscale), _p(mshift), _p(y), _p(mean), _p(invstd), _p(dpre), _p(partial), stream_ptr())
    if _timer is not None:
        _timer.wrap("dgrad", g.flops(), call, *args,
                    nbytes=_nbytes(dy, w_crsk, dx_add, zmask, mask_bits, y, dpre))
        return
    call(*args)


def conv_wgrad_workspace_bytes(g: ConvGeom, max_workgroups: int = 0) -> int:
    """Workspace of conv_wgrad(g, ..., max_workgroups) (0: the full-chip grid)."""
    key = ("ws", g, int(max_workgroups), _plan_env())
    v = _plan_cache.get(key)
    if v is None:
        v = _plan_cache[key] = int(_lib.lib().ssip_conv_wgrad_workspace_bytes_budget(g.desc(), int(max_workgroups)))
    return v


def conv_wgrad(g: ConvGeom, dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, accumulate: bool,
               workspace: torch.Tensor, max_workgroups: int = 0) -> None:
    """max_workgroups > 0: the split-K grid of a wgrad sharing the chip with
    another stream (ssip_conv_wgrad_budget); 0: the full-chip grid."""
    assert dy.numel() == g.N * g.P * g.Q * g.K and x.numel() == g.N * g.H * g.W * g.C
    assert dw.dtype == torch.float32 and dw.numel() == g.K * g.c_real * g.R * g.s_real
    nbytes = workspace.numel() * workspace.element_size()
    if max_workgroups > 0:
        args = ("ssip_conv_wgrad_budget", g.desc(), dtype_code(dy), _p(dy), _p(x), _p(dw), g.c_real, g.s_real,
                int(accumulate), _p(workspace), nbytes, int(max_workgroups), stream_ptr())
    else:
        args = ("ssip_conv_wgrad", g.desc(), dtype_code(dy), _p(dy), _p(x), _p(dw), g.c_real, g.s_real,
                int(accumulate), _p(workspace), nbytes, stream_ptr())
    if _timer is not None:
        # accumulate: dw is read as well as written
        _timer.wrap("wgrad", g.flops(), call, *args, nbytes=_nbytes(dy, x, dw) + (dw.numel() * 4 if accumulate else 0))
        return
    call(*args)


def conv_bnrelu_in_supported(g: ConvGeom, dtype: torch.dtype) -> bool:
    """The conv can take relu(bn(y)) of the layer below as its input, formed in
    its LDS tile (the layer-1 halo geometry; ssip_conv_*_bnrelu_in)."""
    key = ("bri", g, dtype, _plan_env())
    v = _plan_cache.get(key)
    if v is None:
        v = _plan_cache[key] = bool(_lib.lib().ssip_conv_bnrelu_in_supported(g.desc(), _DT[dtype]))
    return v


def conv_fwd_bnrelu_in(g: ConvGeom, y_in: torch.Tensor, in_scale: torch.Tensor, in_shift: torch.Tensor,
                       w_krsc: torch.Tensor, y: torch.Tensor, partial: Optional[torch.Tensor],
                       z_out: Optional[torch.Tensor] = None) -> None:
    """conv_fwd(g, relu(y_in * in_scale + in_shift), w_krsc, y, partial) without
    a separate BN+ReLU pass (bit-identical to bn_apply + conv_fwd); z_out
    (optional, y_in's shape) receives the BN+ReLU output itself, written by the
    conv as it forms its tiles."""
    assert y_in.numel() == g.N * g.H * g.W * g.C and y.numel() == g.N * g.P * g.Q * g.K
    assert in_scale.dtype == torch.float32 and in_scale.numel() == g.C and in_shift.numel() == g.C
    assert z_out is None or (z_out.numel() == y_in.numel() and z_out.dtype == y_in.dtype)
    args = ("ssip_conv_fwd_bnrelu_in", g.desc(), dtype_code(y_in), _p(y_in), _p(in_scale), _p(in_shift), _p(w_krsc),
            _p(y), _p(partial), _p(z_out), stream_ptr())
    if _timer is not None:
        _timer.wrap("fwd", g.flops(), call, *args, nbytes=_nbytes(y_in, w_krsc, y))
        return
    call(*args)


def conv_wgrad_bnrelu_in(g: ConvGeom, dy: torch.Tensor, y_in: torch.Tensor, in_scale: torch.Tensor,
                         in_shift: torch.Tensor, dw: torch.Tensor, accumulate: bool, workspace: torch.Tensor,
                         max_workgroups: int = 0) -> None:
    """conv_wgrad with the input relu(y_in * in_scale + in_shift) formed in LDS."""
    assert dy.numel() == g.N * g.P * g.Q * g.K and y_in.numel() == g.N * g.H * g.W * g.C
    assert dw.dtype == torch.float32 and dw.numel() == g.K * g.C * g.R * g.S
    nbytes = workspace.numel() * workspace.element_size()
    args = ("ssip_conv_wgrad_bnrelu_in", g.desc(), dtype_code(dy), _p(dy), _p(y_in), _p(in_scale), _p(in_shift),
            _p(dw), int(accumulate), _p(workspace), nbytes, int(max_workgroups), stream_ptr())
    if _timer is not None:
        _timer.wrap("wgrad", g.flops(), call, *args, nbytes=_nbytes(dy, y_in, dw) + (dw.numel() * 4 if accumulate else 0))
        return
    call(*args)


def conv_kernel_name(mode: str, g: ConvGeom, dtype: torch.dtype, max_workgroups: int = 0) -> str:
    """The kernel ssip_conv_{fwd,dgrad,wgrad} selects for g (include/ssip.h);
    max_workgroups: ssip_conv_wgrad_budget's choice under that budget."""
    buf = ctypes.create_string_buffer(160)
    call("ssip_conv_kernel_name_budget", {"fwd": 0, "dgrad": 1, "wgrad": 2}[mode], g.desc(), _DT[dtype],
         int(max_workgroups), buf, 160)
    return buf.value.decode()


def stem_bwd_wgrad_supported(g: ConvGeom, dtype: torch.dtype) -> bool:
    return bool(_lib.lib().ssip_stem_bwd_wgrad_supported(g.desc(), _DT[dtype]))


def stem_bwd_wgrad(g: ConvGeom, dpool, idx, y, x, scale, shift, coef, dw, accumulate: bool, workspace) -> None:
    """Stem wgrad with the BN-backward apply formed on the fly (include/ssip.h)."""
    nbytes = workspace.numel() * workspace.element_size()
    args = ("ssip_stem_bwd_wgrad", g.desc(), dtype_code(y), _p(dpool), _p(idx), _p(y), _p(x), _p(scale), _p(shift),
            _p(coef), _p(dw), g.c_real, g.s_real, int(accumulate), _p(workspace), nbytes, stream_ptr())
    if _timer is not None:
        _timer.wrap("wgrad", g.flops(), call, *args, nbytes=_nbytes(dpool, idx, y, x, dw))
        return
    call(*args)


def weight_prep_batch(items, dtype: torch.dtype) -> None:
    """items: [(w_kcrs fp32, Cp, Sp, krsc or None, crsk or None[, kscale fp32 [K] or None])]
    -> one launch per 32 (kscale: per-output-channel factor, a folded eval BN)."""
    for i in range(0, len(items), _lib.WPREP_MAX):
        chunk = items[i:i + _lib.WPREP_MAX]
        arr = (_lib.WPrep * len(chunk))()
        for j, item in enumerate(chunk):
            w, Cp, Sp, krsc, crsk = item[:5]
            ksc = item[5] if len(item) > 5 else None
            assert w.dtype == torch.float32 and w.is_contiguous()
            K, C, R, S = w.shape
            if krsc is not None:
                assert krsc.dtype == dtype and krsc.numel() == K * R * Sp * Cp
            if crsk is not None:
                assert crsk.dtype == dtype and crsk.numel() == K * R * Sp * Cp
            if ksc is not None:
                assert ksc.dtype == torch.float32 and ksc.numel() == K
            arr[j] = _lib.WPrep(K, C, R, S, Cp, Sp, _p(w), _p(krsc), _p(crsk), _p(ksc))
        call("ssip_weight_prep_batch", _DT[dtype], len(chunk), arr, stream_ptr())


def weight_prep(w: torch.Tensor, dtype: torch.dtype, Cp: int, Sp: int, krsc: Optional[torch.Tensor],
                crsk: Optional[torch.Tensor]) -> None:
    K, C, R, S = w.shape
    call("ssip_weight_prep", _DT[dtype], K, C, R, S, Cp, Sp, _p(w), _p(krsc), _p(crsk), stream_ptr())


# ---------------------------------------------------------------------------
# batch norm
# ---------------------------------------------------------------------------
def bn_finalize_scratch_floats(C: int, tiles: int) -> int:
    """floats ssip_bn_finalize's split pass needs behind C*tiles*3 records"""
    n = int(_lib.lib().ssip_bn_finalize_scratch_floats(C, tiles))
    if n < 0:
        raise ValueError(f"bn_finalize_scratch_floats: bad arguments C={C} tiles={tiles}")
    return n


def bn_finalize(C: int, tiles: int, partial, gamma, beta, running_mean, running_var, momentum: float, eps: float,
                update_running: bool, mean, invstd, scale, shift) -> None:
    call("ssip_bn_finalize", C, tiles, _p(partial), _p(gamma), _p(beta), _p(running_mean), _p(running_var),
         float(momentum), float(eps), int(update_running), _p(mean), _p(invstd), _p(scale), _p(shift), stream_ptr())


def bn_eval_coeffs(C: int, gamma, beta, running_mean, running_var, eps: float, mean, invstd, scale, shift) -> None:
    call("ssip_bn_eval_coeffs", C, _p(gamma), _p(beta), _p(running_mean), _p(running_var), float(eps), _p(mean),
         _p(invstd), _p(scale), _p(shift), stream_ptr())


def bn_apply(M: int, C: int, y, scale, shift, residual, relu: bool, z, mbits=None) -> None:
    """mbits: uint8 [M*C/8] receives the ReLU mask (bit j of byte i = z[8i+j] > 0)."""
    call("ssip_bn_apply", dtype_code(y), M, C, _p(y), _p(scale), _p(shift), _p(residual), int(relu), _p(z),
         _p(mbits), stream_ptr())


def bn_apply2(M: int, C: int, y, scale, shift, y2, scale2, shift2, relu: bool, z, mbits=None) -> None:
    """z = relu(y*scale + shift + y2*scale2 + shift2) (block output with a downsample BN residual)."""
    call("ssip_bn_apply2", dtype_code(y), M, C, _p(y), _p(scale), _p(shift), _p(y2), _p(scale2), _p(shift2),
         int(relu), _p(z), _p(mbits), stream_ptr())


def bn_bwd_dual_partial_floats(M: int, C: int) -> int:
    n = int(call("ssip_bn_bwd_dual_partial_floats", M, C))
    if n < 0:
        raise RuntimeError(f"ssip_bn_bwd_dual_partial_floats({M}, {C}) unsupported")
    return n


def bn_bwd_dual(M: int, C: int, dz, zmask, ya, mean_a, invstd_a, gamma_a, dgamma_a, dbeta_a, yb, mean_b, invstd_b,
                gamma_b, dgamma_b, dbeta_b, accumulate: bool, dy_a, dy_b, partial, coef, mbits=None) -> None:
    """Backward of z = relu(BN_a(ya) + BN_b(yb)) (ssip_bn_bwd_dual); coef: 6*C floats.
    The ReLU mask comes from zmask (z > 0) or, when zmask is None, from mbits."""
    call("ssip_bn_bwd_dual", dtype_code(dz), M, C, _p(dz), _p(zmask), _p(mbits), _p(ya), _p(mean_a), _p(invstd_a), _p(gamma_a),
         _p(dgamma_a), _p(dbeta_a), _p(yb), _p(mean_b), _p(invstd_b), _p(gamma_b), _p(dgamma_b), _p(dbeta_b),
         int(accumulate), _p(dy_a), _p(dy_b), _p(partial), _p(coef), stream_ptr())


def bn_bwd_partial_floats(M: int, C: int) -> int:
    return int(_lib.lib().ssip_bn_bwd_partial_floats(M, C))


def bn_bwd(M: int, C: int, dz, zmask, y, mean, invstd, gamma, dgamma, dbeta, accumulate: bool, dy, dpre, partial,
           coef, mbits=None) -> None:
    """ReLU mask from zmask (z > 0) or, when zmask is None, from mbits (ssip_bn_apply's mask bits)."""
    call("ssip_bn_bwd", dtype_code(dz), M, C, _p(dz), _p(zmask), _p(mbits), _p(y), _p(mean), _p(invstd), _p(gamma),
         _p(dgamma), _p(dbeta), int(accumulate), _p(dy), _p(dpre), _p(partial), _p(coef), stream_ptr())


def bn_relu_bwd(M: int, C: int, dz, y, mean, invstd, scale, shift, gamma, dgamma, dbeta, accumulate: bool, dy,
                partial, coef) -> None:
    """BN+ReLU backward with the mask recomputed from y (no z read)."""
    call("ssip_bn_relu_bwd", dtype_code(dz), M, C, _p(dz), _p(y), _p(mean), _p(invstd), _p(scale), _p(shift),
         _p(gamma), _p(dgamma), _p(dbeta), int(accumulate), _p(dy), _p(partial), _p(coef), stream_ptr())


def bn_bwd_from_partials(M: int, C: int, tiles: int, partial, dout, y, mean, invstd, gamma, dgamma, dbeta,
                         accumulate: bool, dy, coef) -> None:
    call("ssip_bn_bwd_from_partials", dtype_code(dout), M, C, tiles, _p(partial), _p(dout), _p(y), _p(mean),
         _p(invstd), _p(gamma), _p(dgamma), _p(dbeta), int(accumulate), _p(dy), _p(coef), stream_ptr())


def stem_bn_pool_fwd(N, H, W, C, k, s, pad, y, scale, shift, out, idx, ymax=None) -> None:
    """maxpool(relu(BN(y))) with argmax bytes, no full-resolution activation;
    ymax (optional, pooled shape): y at each window's argmax, for the backward."""
    call("ssip_stem_bn_pool_fwd", dtype_code(y), N, H, W, C, k, s, pad, _p(y), _p(scale), _p(shift), _p(out),
         _p(idx), _p(ymax), stream_ptr())


def stem_bn_pool_kernel_name(dtype: torch.dtype, N, H, W, C, k, s, pad, has_ymax: bool) -> str:
    """The kernel stem_bn_pool_fwd launches for this shape (ssip_stem_bn_pool_kernel_name, ABI 14)."""
    buf = ctypes.create_string_buffer(96)
    call("ssip_stem_bn_pool_kernel_name", _DT[dtype], N, H, W, C, k, s, pad, int(has_ymax), buf, 96)
    return buf.value.decode()


def stem_pool_bn_bwd_partial_floats(N, H, W, C) -> int:
    return int(_lib.lib().ssip_stem_pool_bn_bwd_partial_floats(N, H, W, C))


def stem_pool_bn_bwd(N, H, W, C, k, s, pad, dpool, idx, y, mean, invstd, scale, shift, gamma, dgamma, dbeta,
                     accumulate: bool, dy, partial, coef, ymax=None) -> None:
    """BN(+ReLU) backward of the stem through the max-pool, one reduction pass
    (over the pooled grid when the forward's ymax is given) and one apply pass
    over y (see include/ssip.h)."""
    call("ssip_stem_pool_bn_bwd", dtype_code(y), N, H, W, C, k, s, pad, _p(dpool), _p(idx), _p(y), _p(ymax), _p(mean),
         _p(invstd), _p(scale), _p(shift), _p(gamma), _p(dgamma), _p(dbeta), int(accumulate), _p(dy), _p(partial),
         _p(coef), stream_ptr())


def relu_bwd(g, z, out) -> None:
    call("ssip_relu_bwd", dtype_code(g), g.numel(), _p(g), _p(z), _p(out), stream_ptr())


# ---------------------------------------------------------------------------
# pooling / head / losses
# ---------------------------------------------------------------------------
def maxpool_fwd(N, H, W, C, k, s, pad, x, y, idx) -> None:
    call("ssip_maxpool_fwd", dtype_code(x), N, H, W, C, k, s, pad, _p(x), _p(y), _p(idx), stream_ptr())


def maxpool_bwd(N, H, W, C, k, s, pad, dy, idx, dx) -> None:
    call("ssip_maxpool_bwd", dtype_code(dy), N, H, W, C, k, s, pad, _p(dy), _p(idx), _p(dx), stream_ptr())


def avgpool_fc_fwd(B, PQ, C, J, z, w, bias, feat, logits) -> None:
    call("ssip_avgpool_fc_fwd", dtype_code(z), B, PQ, C, J, _p(z), _p(w), _p(bias), _p(feat), _p(logits),
         stream_ptr())


def avgpool_fc_bwd(dtype: torch.dtype, B, PQ, C, J, dlogits, w, feat, dz, dw, dbias, accumulate: bool) -> None:
    call("ssip_avgpool_fc_bwd", _DT[dtype], B, PQ, C, J, _p(dlogits), _p(w), _p(feat), _p(dz), _p(dw), _p(dbias),
         int(accumulate), stream_ptr())


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, grad_scale: float = 1.0, want_grad: bool = True):
    """Returns (loss[1], dlogits or None, pred[B]) — all device tensors."""
    B, J = logits.shape
    logits = logits.contiguous().float()
    labels = labels.contiguous().to(torch.int64)
    loss = torch.empty(1, device=logits.device, dtype=torch.float32)
    dl = torch.empty_like(logits) if want_grad else None
    pred = torch.empty(B, device=logits.device, dtype=torch.int64)
    call("ssip_cross_entropy", B, J, _p(logits), _p(labels), float(grad_scale), _p(loss), _p(dl), _p(pred),
         stream_ptr())
    return loss, dl, pred


def semi_loss(zl, yl, zw, zs, tau: float, lambda_u: float, dz: Optional[torch.Tensor] = None):
    """dz (optional): one [Bl+Bu, J] buffer receiving [dzl; dzs] (the joint
    forward's logit gradient, written in place: no concatenation pass)."""
    Bl = 0 if zl is None else zl.shape[0]
    Bu = 0 if zw is None else zw.shape[0]
    J = (zl if zl is not None else zw).shape[1]
    dev = (zl if zl is not None else zw).device
    out = torch.empty(4, device=dev, dtype=torch.float32)
    if dz is not None:
        assert dz.shape == (Bl + Bu, J) and dz.dtype == torch.float32 and dz.is_contiguous()
        dzl = dz[:Bl] if zl is not None else None
        dzs = dz[Bl:] if zs is not None else None
    else:
        dzl = torch.empty_like(zl) if zl is not None else None
        dzs = torch.empty_like(zs) if zs is not None else None
    pseudo = torch.empty(Bu, device=dev, dtype=torch.int64) if Bu else None
    mask = torch.empty(Bu, device=dev, dtype=torch.uint8) if Bu else None
    call("ssip_semi_loss", Bl, Bu, J, _p(zl), _p(yl), _p(zw), _p(zs), float(tau), float(lambda_u), _p(out), _p(dzl),
         _p(dzs), _p(pseudo), _p(mask), stream_ptr())
    return out, dzl, dzs, pseudo, mask


def softmax_select(logits: torch.Tensor, threshold: float = 0.0, pos_col: int = 0):
    """softmax, max, argmax, (max >= threshold), P(pos_col) in one launch."""
    B, J = logits.shape
    logits = logits.contiguous().float()
    dev = logits.device
    probs = torch.empty_like(logits)
    conf = torch.empty(B, device=dev, dtype=torch.float32)
    pred = torch.empty(B, device=dev, dtype=torch.int64)
    keep = torch.empty(B, device=dev, dtype=torch.uint8)
    pos = torch.empty(B, device=dev, dtype=torch.float32)
    call("ssip_softmax_select", B, J, _p(logits), float(threshold), int(pos_col), _p(probs), _p(conf), _p(pred),
         _p(keep), _p(pos), stream_ptr())
    return probs, conf, pred, keep, pos


def adamw(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0) -> None:
    call("ssip_adamw", param.numel(), _p(param), _p(grad), _p(exp_avg), _p(exp_avg_sq), float(lr), float(beta1),
         float(beta2), float(eps), float(weight_decay), int(step), float(grad_scale), stream_ptr())


def adamw_sched_step(sched: torch.Tensor, beta1: float, beta2: float) -> None:
    assert sched.dtype == torch.float64 and sched.numel() >= 7
    call("ssip_adamw_sched_step", _p(sched), float(beta1), float(beta2), stream_ptr())


def adamw_dev(param, grad, exp_avg, exp_avg_sq, sched, beta1, beta2, eps, weight_decay, grad_scale=1.0,
              advance: bool = False) -> None:
    """advance: this launch also advances the device schedule (t, bias
    corrections) -- the first update launch of a step; sched needs 7 slots
    (ABI 11: 5-6 stage the next step's bias corrections, 0 = not staged)."""
    assert sched.dtype == torch.float64 and sched.numel() >= (7 if advance else 4)
    call("ssip_adamw_dev", param.numel(), _p(param), _p(grad), _p(exp_avg), _p(exp_avg_sq), _p(sched), float(beta1),
         float(beta2), float(eps), float(weight_decay), float(grad_scale), int(bool(advance)), stream_ptr())


def nchw_to_nhwc(x: torch.Tensor, Cp: int, dtype: torch.dtype, pad: int = 0) -> torch.Tensor:
    """f32 NCHW -> [B, H+2*pad, W+2*pad, Cp] with a zero border and zero channel padding."""
    B, C, H, W = x.shape
    x = x.contiguous().float()
    out = torch.empty((B, H + 2 * pad, W + 2 * pad, Cp), device=x.device, dtype=dtype)
    call("ssip_nchw_to_nhwc", _DT[dtype], B, C, H, W, Cp, pad, _p(x), _p(out), stream_ptr())
    return out
