"""Per-phase cycle counts of k_list_pack on virtual ranks (experiment tool; run
on the GPU box with a variant library built with -DGP_LP_STAMPS=1).

    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_lpst.so python tools/pack_stamps.py <n> <W> <rounds>

Imp3D push-sum, activation pre-roll, then `rounds` steady rounds; prints the mean
s_memtime cycles per pack block of each phase (gp_debug_lp_stamps, gp_xchg.hip).
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n, W, rounds = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    from gossipprotocol_amd import Simulation
    s = Simulation(n, "Imp3D", "push-sum", virtual_ranks=W, experimental=True)
    L = s._L
    fn = L.gp_debug_lp_stamps
    fn.argtypes = [C.POINTER(C.c_double), C.c_int]
    buf = (C.c_double * 8)()
    while s.info().active < s.population:
        s.step(8)
    s.sync()
    fn(buf, 1)
    s.step(rounds)
    s.sync()
    fn(buf, 1)
    names = ["lds init", "wave 0 tile: loads, bitmap, scans", "wait for the block's tiles", "reservations",
             "wave 0 header words", "wave 0 headers + payloads"]
    for q, nm in enumerate(names):
        print("%-36s %10.0f cycles" % (nm, buf[q]))
    print("%-36s %10.0f" % ("blocks", buf[6]))
    s.close()


if __name__ == "__main__":
    main()
