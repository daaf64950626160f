"""CPU-side checks of the drop-in boundary: libnetty_amd.so loads and exports every entry point
include/netty_amd.h declares (no compute calls: there is no GPU here)."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "netty_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(nx_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_header_declares_entry_points():
    names = _declared()
    for must in ("nx_snappy_encode_batch", "nx_snappy_decode_batch", "nx_crc32c_masked_batch", "nx_fastlz_compress_batch",
                 "nx_fastlz_decompress_batch", "nx_lzf_encode_batch", "nx_lzf_decode_batch",
                 "nx_snappy_frame_encoder_encode", "nx_snappy_frame_decoder_decode"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from netty_amd import _lib
    L = _lib.load()
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert not missing, missing
    # every ctypes signature in _lib.py is a declared symbol too
    assert set(_lib.EXPORTED) <= set(_declared())


def test_exports_are_c_abi_symbols():
    so = os.path.join(ROOT, "netty_amd", "libnetty_amd.so")
    out = subprocess.check_output(["nm", "-D", "--defined-only", so], text=True)
    syms = {l.split()[-1] for l in out.splitlines() if l.strip()}
    for n in _declared():
        assert n in syms, n  # unmangled extern "C"


def test_host_only_calls_without_gpu():
    from netty_amd import _lib
    L = _lib.load()
    assert L.nx_snappy_max_compressed_length(65536) == 32 + 65536 + 65536 // 6
    assert _lib.status_string(-2) == "Offset is less than minimum permissible value"
    assert b"gfx950" in L.nx_version()


def test_product_has_no_oracle_dependency():
    # the product package must never import or link the oracle (checker only)
    pkg = os.path.join(ROOT, "netty_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".hpp", ".h")):
                txt = open(os.path.join(dirpath, f), errors="ignore").read()
                assert not re.search(r"^\s*(import|from)\s+oracle|pyoracle|#\s*include\s*[<\"].*oracle|liboracle", txt,
                                     flags=re.M), f
    out = subprocess.check_output(["ldd", os.path.join(pkg, "libnetty_amd.so")], text=True)
    assert "oracle" not in out


def test_one_decode_path_no_environment_kernel_selection():
    """the library's kernel choice never depends on the environment.  The only
    getenv calls left in netty_amd/csrc are diagnostics (error text, a fault trace, scan statistics)."""
    allowed = {"NX_HIP_DEBUG", "NX_SEGV_TRACE", "NX_SCAN_STATS"}
    src = os.path.join(ROOT, "netty_amd", "csrc")
    seen = set()
    for f in os.listdir(src):
        txt = open(os.path.join(src, f), errors="ignore").read()
        for name in re.findall(r'getenv\("([A-Z0-9_]+)"\)', txt):
            seen.add(name)
            assert name in allowed, (f, name)
    assert "NX_EXPANDER" not in seen and "NX_DECODE_MODE" not in seen
    for f in ("expand_units.hpp", "expand_frame.hpp"):
        assert not os.path.exists(os.path.join(src, f))


def _plan(n, slots=327680, cus=256):
    import ctypes
    from netty_amd import _lib
    L = _lib.load()
    sizes = (ctypes.c_uint32 * 256)()
    cnt = ctypes.c_uint32(0)
    assert L.nx_snappy_encode_plan_for(n, slots, cus, sizes, 256, ctypes.byref(cnt)) == 0
    return [sizes[i] for i in range(cnt.value)]


def test_encode_launch_plan_host_arithmetic():
    """The Snappy encoder's launch plan (round 6), host-only: k = ceil(n / slots) launches,
    equal in steps of half a block per CU, the rest below one step on the last, never above the slots."""
    assert _plan(1638400) == [327680] * 5  # N = 1 of the 100 GiB job
    assert _plan(819200) == [294912, 262144, 262144]  # N = 2
    assert _plan(409600) == [196608, 212992]  # N = 4
    assert _plan(204800) == [204800]  # N = 8
    assert _plan(1048576) == [262144] * 4  # the weak 1 M field
    assert _plan(0) == [] and _plan(1) == [1]
    import random
    rng = random.Random(5)
    for _ in range(2000):
        cus = rng.choice((64, 80, 256, 304))
        slots = rng.choice((cus * 1280, cus * 1024, 65536, 20480, 16640, 100 * 256))
        n = rng.randrange(1, 3_000_000)
        p = _plan(n, slots, cus)
        assert sum(p) == n and max(p) <= slots and len(p) == -(-n // slots), (n, slots, cus, p)
        if len(p) > 1:  # equal launches: within one step (+ the last launch's rest), or a plain equal split
            assert max(p) - min(p) <= 2 * cus * 128 or max(p) - min(p) <= -(-n // len(p)), (n, slots, cus, p)
