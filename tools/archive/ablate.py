"""Build variants of the round kernels and time them (experiment tool, not part
of the product).

    python tools/ablate.py build            # CPU: compile variants into build/ablate/
    python tools/ablate.py run [n] [names]  # GPU: steady-state ms/round of each variant

Each variant compiles gp_round.hip of the experiments build (-DGP_EXPERIMENTS)
with extra -D flags (the knobs at the top of gp_round.hip) and links it with
the other experiments objects (build/obj_exp, made by the csrc Makefile).
ABLATE_ONLY=a,b limits the build to some variants.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gossipprotocol_amd", "csrc")
OUT = os.path.join(ROOT, "build", "ablate")
OBJ = os.path.join(ROOT, "build", "obj_exp")
VARIANTS = {  # name -> extra -D flags for gp_round.hip
    "base": [],
    "stamps": ["-DGP_STAMPS=1"],
    "nofma": ["-DGP_FMA_FOLD=0"],
    "noz": ["-DGP_ABL_DIRS=48"],
    "nox": ["-DGP_ABL_DIRS=3"],
    "noy": ["-DGP_ABL_DIRS=12"],
    "nolat": ["-DGP_ABL_DIRS=63"],
    "n2m6": ["-DGP_NPT=2", "-DGP_MINB=6"],
    "n2m5": ["-DGP_NPT=2", "-DGP_MINB=5"],
    "minb4": ["-DGP_MINB=4"],
    "minb6": ["-DGP_MINB=6"],
    "npt2": ["-DGP_NPT=2"],
    "plainld": ["-DGP_NT_LOADS=0"],
    "plainst": ["-DGP_NT_STORES=0"],
    "nozdpp": ["-DGP_ZDPP=0"],
    "t512m6": ["-DGP_TPB=512", "-DGP_NPT=2", "-DGP_MINB=6"],
    "t1024m8": ["-DGP_TPB=1024", "-DGP_NPT=1", "-DGP_MINB=8"],
    "prio0": ["-DGP_SETPRIO=0"],
    "prio1": ["-DGP_SETPRIO=1"],
    "prio2": ["-DGP_SETPRIO=2"],
    "prio3": ["-DGP_SETPRIO=3"],
    "prio4": ["-DGP_SETPRIO=4"],
    "prio5": ["-DGP_SETPRIO=5"],
    "prio3v1": ["-DGP_SETPRIO=3", "-DGP_PRIO=1"],
    "prio3v3": ["-DGP_SETPRIO=3", "-DGP_PRIO=3"],
    "ng2m4": ["-DGP_NG=2", "-DGP_MINB=4"],
    "steal": ["-DGP_STEAL=1"],
    "sched0": ["-DGP_SETPRIO=0", "-DGP_STEAL=0"],
    "minb6p": ["-DGP_MINB=6"],
}
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-DGP_EXPERIMENTS"]


def build():
    os.makedirs(OUT, exist_ok=True)
    only = os.environ.get("ABLATE_ONLY")
    names = only.split(",") if only else list(VARIANTS)
    procs = []
    for name in names:
        obj = os.path.join(OUT, f"gp_round_{name}.o")
        cmd = ["/opt/rocm/bin/hipcc", *FLAGS, *VARIANTS[name], "-c", "-o", obj, os.path.join(CSRC, "gp_round.hip")]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        assert p.wait() == 0
    others = [os.path.join(OBJ, f) for f in sorted(os.listdir(OBJ)) if f.endswith(".o") and f != "gp_round.o"]
    for name in names:
        so = os.path.join(OUT, f"lib_{name}.so")
        subprocess.check_call(["/opt/rocm/bin/hipcc", *FLAGS, "-shared", "-o", so, *others,
                               os.path.join(OUT, f"gp_round_{name}.o"), "-L/opt/rocm/lib", "-lrccl"])


def run(n, only=None):
    res = {}
    topo = os.environ.get("ABLATE_TOPO", "Imp3D")
    for name in (only or VARIANTS):
        so = os.path.join(OUT, f"lib_{name}.so")
        code = ("import sys,json; sys.path.insert(0,%r)\n"
                "from gossipprotocol_amd import Simulation\n"
                "s=Simulation(%d,%r,'push-sum',kernel_timing=True,experimental=True)\n"
                "P=s.population\n"
                "pre=0\nwhile s.info().active < P and pre < 300: pre += len(s.step(8))\n"
                "import ctypes as C\nL=s._L\nst=hasattr(L,'gp_debug_stamps')\nbuf=(C.c_double*8)()\n"
                "s.sync()\nif st: L.gp_debug_stamps(buf,1)\n"
                "s.kernel_stats(reset=True); s.step(10); s.sync()\n"
                "if st: L.gp_debug_stamps(buf,1); print('stamps', [round(buf[q]) for q in range(7)], file=sys.stderr)\n"
                "ms,k,_=s.kernel_stats(); print(json.dumps(ms/k))\n") % (ROOT, n, topo)
        env = dict(os.environ, GOSSIP_HIP_LIB_EXPERIMENT=so)
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode:
            print(name, "FAILED", out.stderr[-500:], flush=True)
            sys.exit(1)
        res[name] = float(out.stdout.strip().splitlines()[-1])
        print(f"{name:14s} {res[name]:8.2f} ms/round", flush=True)
        for line in out.stderr.splitlines():
            if line.startswith("stamps"):
                print(f"{'':14s} {line}  (cycles/tile: in-edge, stage issue, stage wait, nodes, dirs, bytes; tiles)",
                      flush=True)
    return res


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 10**9, sys.argv[3].split(",") if len(sys.argv) > 3 else None)
