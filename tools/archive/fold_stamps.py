"""Per-phase cycle counts of the fused full-topology fold (experiment tool; run on
the GPU box with a variant library built with -DGP_FB_STAMPS=1).

    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_fbst.so python tools/fold_stamps.py <n> <rounds>

Full push-sum on one rank: 48 rounds of pre-roll, then `rounds` rounds; prints the
mean s_memtime cycles per tile of each k_fb_fold<true> phase (gp_debug_fb_stamps).
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n, rounds = int(sys.argv[1]), int(sys.argv[2])
    from gossipprotocol_amd import Simulation
    s = Simulation(n, "full", "push-sum", experimental=True)
    fn = s._L.gp_debug_fb_stamps
    fn.argtypes = [C.POINTER(C.c_double), C.c_int]
    buf = (C.c_double * 8)()
    s.step(48)
    s.sync()
    fn(buf, 1)
    s.step(rounds)
    s.sync()
    fn(buf, 1)
    names = ["loads issued, Philox, receiver counts", "scan, messages to LDS", "sort, fold, ratio, state out",
             "send: counts, reserve, scatter", "send: write-out"]
    for q, nm in enumerate(names):
        print("%-40s %10.0f cycles" % (nm, buf[q]))
    print("%-40s %10.0f" % ("tiles", buf[5]))
    s.close()


if __name__ == "__main__":
    main()
