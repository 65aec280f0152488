"""CPU: the C-ABI library loads and exports every symbol include/ssip.h
declares (no compute calls without a GPU)."""
import re
from pathlib import Path

from ssip import _lib

ROOT = Path(__file__).resolve().parents[1]


def test_header_and_binding_agree():
    hdr = (ROOT / "include" / "ssip.h").read_text()
    declared = set(re.findall(r"^\s*(?:const char\*|int64_t|int|void|ssip_plan\*)\s+(ssip_\w+)\(", hdr, re.M))
    assert declared == set(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_symbol():
    lib = _lib.lib()
    for name in _lib.EXPORTED_SYMBOLS:
        assert hasattr(lib, name), name
    assert lib.ssip_version() == _lib.abi_version_expected() == _lib.ABI_VERSION


def test_build_entry_checks_the_header_version():
    # __graft_entry__.build() compares ssip_version() against the header's
    # SSIP_ABI_VERSION (not a literal): both must agree with the built library
    hdr = (ROOT / "include" / "ssip.h").read_text()
    v = int(re.search(r"^#define\s+SSIP_ABI_VERSION\s+(\d+)", hdr, re.M).group(1))
    assert _lib.abi_version_expected() == v == _lib.lib().ssip_version()
    src = (ROOT / "__graft_entry__.py").read_text()
    assert "abi_version_expected()" in src


def test_plan_thunks_match_the_header():
    """csrc/plan_thunks.inc (the typed replay thunks) is generated from
    include/ssip.h and committed: it must be current."""
    import subprocess
    import sys

    rc = subprocess.run([sys.executable, str(ROOT / "tools" / "gen_plan_thunks.py"), "--check"]).returncode
    assert rc == 0, "run tools/gen_plan_thunks.py"


def test_plan_api_records_without_a_device():
    """A plan can be built and inspected on the host (recording a call only
    copies its slots and blobs; nothing is launched until ssip_plan_run)."""
    import ctypes

    lib = _lib.lib()
    h = lib.ssip_plan_create()
    try:
        fi = lib.ssip_plan_fn_index(b"ssip_counters_add")
        assert fi >= 0 and lib.ssip_plan_fn_index(b"ssip_version") == -1
        slots = (ctypes.c_uint64 * 4)(3, 0, 1, 0)
        blob = (ctypes.c_void_p * 3)(16, 32, 48)
        lens = (ctypes.c_int64 * 4)(0, ctypes.sizeof(blob), 0, 0)
        assert lib.ssip_plan_add_call(h, fi, 4, slots, lens, blob) == 0
        assert lib.ssip_plan_add_call(h, fi, 3, slots, lens, blob) == -1  # wrong arity
        assert lib.ssip_plan_add_marker(h) == 1
        assert lib.ssip_plan_segments(h) == 2 and lib.ssip_plan_num_ops(h) == 1
        assert lib.ssip_plan_run(h, 5) == -1
    finally:
        lib.ssip_plan_destroy(h)


def test_argument_errors_surface_as_status_codes():
    lib = _lib.lib()
    d = _lib.ConvDesc(1, 8, 8, 24, 64, 3, 3, 1, 1, 8, 8)  # C=24 is not a multiple of 32
    assert lib.ssip_conv_fwd_partial_floats(d) < 0
    rc = lib.ssip_conv_fwd(d, 0, None, None, None, None, None)
    assert rc == -1
    assert b"multiple of 32" in lib.ssip_last_error()


def test_product_never_imports_the_oracle():
    pkg = ROOT / "semi-supervised-image-processing_amd"
    for f in list(pkg.rglob("*.py")) + list(pkg.rglob("*.hip")) + list(pkg.rglob("*.cpp")):
        txt = f.read_text()
        assert "import oracle" not in txt and "from oracle" not in txt, f
