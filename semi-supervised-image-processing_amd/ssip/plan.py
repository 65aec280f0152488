"""Launch plans: record one eager step, replay it from C++ (csrc/plan.cpp).

Recording runs the ordinary Python engine once with a `PlanRecorder`
installed in ``ssip._lib``: every stream-ordered C-ABI call executes as usual
AND is appended to the plan with its exact arguments; every tensor whose
device pointer is taken (``_lib.ptr``) is kept alive by the plan, so the
addresses a replay uses stay valid and private to it.  Stream hand-offs made
through ``ops.wait_stream`` become event record / wait pairs, and host work
that must run at replay time too (collective launches from the gradient
bucketer) goes through ``ops.host_callback``: it ends a plan segment, and a
replay calls it between ``ssip_plan_run`` of consecutive segments.

Contract of a recorded region (what makes a replay equal to a fresh eager
step): every device-side effect must come from a C-ABI call or an
``ops.host_callback``; host-side state changed inside the region (Python
objects, torch allocator) is not replayed.  ssip's train step keeps to it:
AdamW runs from its device-side schedule, the BN batch counters advance with
``ssip_counters_add``, the loss writes its logit gradients into one buffer.
"""
from __future__ import annotations

import ctypes
import struct
from typing import Any, Callable, List, Optional, Tuple

from . import _lib


class PlanRecorder:
    def __init__(self, plan: "Plan"):
        self.plan = plan
        self.keep = plan.keep

    def on_call(self, name: str, args) -> None:
        lib = _lib.lib()
        fi = self.plan.fn_index(name)
        if fi < 0:
            return  # queries / non-stream entry points are not part of a launch sequence
        argtypes = _lib._SIGS[name][1]
        n = len(args)
        slots = (ctypes.c_uint64 * n)()
        lens = (ctypes.c_int64 * n)()
        blob = bytearray()
        for i, (a, t) in enumerate(zip(args, argtypes)):
            if isinstance(a, (ctypes.Structure, ctypes.Array)):
                b = ctypes.string_at(ctypes.addressof(a), ctypes.sizeof(a))
                lens[i] = len(b)
                blob += b
            elif a is None:
                slots[i] = 0
            elif t is ctypes.c_float:
                slots[i] = struct.unpack("<I", struct.pack("<f", float(a)))[0]
            elif t is ctypes.c_double:
                slots[i] = struct.unpack("<Q", struct.pack("<d", float(a)))[0]
            else:
                slots[i] = int(a) & 0xFFFFFFFFFFFFFFFF
        data = (ctypes.c_uint8 * max(1, len(blob))).from_buffer_copy(bytes(blob) or b"\0")
        _lib.check(lib.ssip_plan_add_call(self.plan.handle, fi, n, slots, lens, data), f"record {name}")

    def wait_stream(self, dst_stream: int, src_stream: int) -> None:
        lib = _lib.lib()
        ev = lib.ssip_plan_add_event(self.plan.handle, src_stream)
        if ev < 0:
            _lib.check(ev, "ssip_plan_add_event")
        _lib.check(lib.ssip_plan_add_wait(self.plan.handle, dst_stream, ev), "ssip_plan_add_wait")

    def callback(self, fn: Callable, args: Tuple) -> None:
        self.plan.callbacks.append((fn, args))
        seg = _lib.lib().ssip_plan_add_marker(self.plan.handle)
        if seg < 0:
            _lib.check(seg, "ssip_plan_add_marker")


class Plan:
    """A recorded launch sequence (see module docstring)."""

    def __init__(self):
        self.handle = _lib.lib().ssip_plan_create()
        if not self.handle:
            raise RuntimeError("ssip_plan_create failed")
        self.keep: List[Any] = []            # tensors whose pointers the plan uses
        self.callbacks: List[Tuple[Callable, Tuple]] = []   # host work between segments
        self._fn = {}

    def fn_index(self, name: str) -> int:
        i = self._fn.get(name)
        if i is None:
            i = self._fn[name] = int(_lib.lib().ssip_plan_fn_index(name.encode()))
        return i

    def __enter__(self) -> "Plan":
        if _lib.RECORDER is not None:
            raise RuntimeError("ssip: a launch plan is already being recorded")
        _lib.RECORDER = PlanRecorder(self)
        return self

    def __exit__(self, *exc) -> None:
        _lib.RECORDER = None

    @property
    def num_ops(self) -> int:
        return int(_lib.lib().ssip_plan_num_ops(self.handle))

    @property
    def segments(self) -> int:
        return int(_lib.lib().ssip_plan_segments(self.handle))

    def replay(self) -> None:
        """Enqueue the whole plan: segment 0, callback 0, segment 1, ..."""
        lib = _lib.lib()
        for seg in range(self.segments):
            rc = lib.ssip_plan_run(self.handle, seg)
            if rc != 0:
                _lib.check(rc, "ssip_plan_run")
            if seg < len(self.callbacks):
                fn, args = self.callbacks[seg]
                fn(*args)

    def close(self) -> None:
        if self.handle:
            _lib.lib().ssip_plan_destroy(self.handle)
            self.handle = None
        self.keep.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def recording() -> Optional[PlanRecorder]:
    return _lib.RECORDER
