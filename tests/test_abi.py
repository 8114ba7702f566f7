"""CPU tests of the drop-in boundary: libgossip_hip.so loads, exports every symbol
include/gossip_hip.h declares, and its host-only entry points behave.  No compute
call is made here (no GPU in this container)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from gossipprotocol_amd import _lib as L
from gossipprotocol_amd import resolve

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gossip_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gp_[a-z_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    names = declared_symbols()
    assert len(names) >= 17
    lib = C.CDLL(L.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(n for n, _, _ in L.SIGNATURES) == names


def test_version_and_parsers():
    lib = L.lib()
    assert lib.gp_version() == 10100
    assert [lib.gp_parse_topology(t) for t in (b"line", b"full", b"3D", b"Imp3D", b"imp3D")] == [0, 1, 2, 3, 3]
    assert lib.gp_parse_topology(b"3d") == -1  # case-sensitive like Program.fs:238
    assert b"unknown topology" in lib.gp_last_error()
    assert lib.gp_parse_algorithm(b"push-sum") == 1 and lib.gp_parse_algorithm(b"gossip") == 0
    assert lib.gp_parse_algorithm(b"push sum") == -1
    assert b"option invalid" in lib.gp_last_error()


def test_resolve_through_abi():
    assert resolve(1000, "line") == (1001, 1000, 0)
    assert resolve(10**9, "imp3D") == (10**9, 10**9, 1000)
    assert resolve(26, "3D") == (27, 27, 3)
    with pytest.raises(L.GossipError):
        resolve(0, "line")
    with pytest.raises(L.GossipError):
        resolve(5 * 10**9, "full")  # beyond 32-bit node ids


def test_struct_layout_matches_c(tmp_path):
    """The P/Invoke / ctypes structs are blittable and match the C layout."""
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "gossip_hip.h"\nint main(void){'
                   'printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(gp_config), offsetof(gp_config, max_rounds),'
                   'sizeof(gp_result), offsetof(gp_result, status), sizeof(gp_info), offsetof(gp_info, topology));'
                   'return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)])
    got = list(map(int, subprocess.check_output([str(exe)]).split()))
    want = [C.sizeof(L.GpConfig), L.GpConfig.max_rounds.offset, C.sizeof(L.GpResult), L.GpResult.status.offset,
            C.sizeof(L.GpInfo), L.GpInfo.topology.offset]
    assert got == want


def test_create_without_gpu_fails_loudly():
    """On a host without gfx950 the product refuses (no CPU fallback)."""
    from gossipprotocol_amd import Simulation
    try:
        sim = Simulation(10, "line", "gossip")
    except L.GossipError as e:
        assert e.code == -6  # GP_ENODEV
        return
    sim.close()  # a GPU is present: creation is allowed


def test_cli_invalid_option():
    exe = os.path.join(ROOT, "gossipprotocol_amd", "gossip")
    r = subprocess.run([exe, "10", "line", "push_sum"], capture_output=True, text=True)
    assert r.returncode == 2 and r.stdout.strip() == "option invalid"
    r = subprocess.run([exe, "10", "ring", "gossip"], capture_output=True, text=True)
    assert r.returncode == 2 and "unknown topology" in r.stderr


def test_population_cap_matches_oracle():
    """GP_MAX_POPULATION (include/gossip_hip.h): the largest P both the product and
    the oracle accept; one more is refused by both (tiles of 1024 ids never wrap)."""
    from tests.oracle_ctypes import lib as olib
    cap = 0xFFFFF000
    assert resolve(cap - 1, "line")[0] == cap
    with pytest.raises(L.GossipError):
        resolve(cap, "line")
    P, T, g = C.c_int64(), C.c_int64(), C.c_int64()
    o = olib()
    o.or_resolve.restype = C.c_int
    o.or_resolve.argtypes = [C.c_int64, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    assert o.or_resolve(cap - 1, 0, C.byref(P), C.byref(T), C.byref(g)) == 0 and P.value == cap
    assert o.or_resolve(cap, 0, C.byref(P), C.byref(T), C.byref(g)) == -1
    assert resolve(1625**3, "Imp3D")[2] == 1625  # the largest lattice edge still fits


def test_product_library_has_no_environment_switches():
    """The product library reads no GP_* environment variable: kernel variants and
    test overrides live only in the experiments build (-DGP_EXPERIMENTS)."""
    prod = open(L.LIB_PATH, "rb").read()
    exp = open(os.path.join(os.path.dirname(L.LIB_PATH), "libgossip_hip_exp.so"), "rb").read()
    for knob in (b"GP_KERNEL", b"GP_XSEGS", b"GP_WALK", b"GP_WX", b"GP_STAGE_CAP", b"GP_NO_PACK",
                 b"GP_FORCE_RCCL", b"GP_XCAP", b"GP_WIDE", b"GP_RQ8", b"GP_CHECK_CLOSE", b"GP_FUSE",
                 b"GP_RREGIONS", b"GP_FB_FUSED", b"GP_IND4_WIDE"):
        assert knob not in prod, knob
        assert knob in exp, knob
    # overrides of variants measured and rejected are gone from both builds (round 6)
    for knob in (b"GP_PSTREAM", b"GP_XREGIONS", b"GP_XHALVES", b"GP_HALO_FULL", b"GP_RLAST", b"GP_FB_S1D",
                 b"GP_FOLD_BLOCKS", b"GP_GRID"):
        assert knob not in prod and knob not in exp, knob
