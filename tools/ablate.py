"""Ablation study of the round kernel (experiment tool, not part of the product).

    python tools/ablate.py build            # CPU: compile variants into build/ablate/
    python tools/ablate.py run [n]           # GPU: time each variant (steady state from round 0)

Each variant compiles gp_round.hip with -DGP_NPT=<n> -DGP_ABLATE=<mask>
(switch meanings at the top of gp_round.hip); ablated results are wrong by
design, only the steady-state time per round matters (the activation pre-roll
uses the variant itself, so heavily ablated variants may activate slowly).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gossipprotocol_amd", "csrc")
OUT = os.path.join(ROOT, "build", "ablate")
# name -> (GP_NPT, GP_ABLATE mask) for gp_round.hip (mask bits at the top of gp_round.hip)
VARIANTS = {  # name -> (NPT, GP_ABLATE mask[, GP_MINB[, GP_TPB[, extra -D flags]]])
    "base_npt4": (4, 0),
    "no_rgather": (4, 1), "no_lgather": (4, 2), "no_inlist": (4, 4), "no_nextdir": (4, 8),
    "no_ephilox": (4, 16), "no_ratio": (4, 64), "no_gathers": (4, 1 | 2),
    "no_xgather": (4, 256), "no_ygather": (4, 512), "no_rfold": (4, 2048), "fake_src": (4, 4096),
    "no_rfold_rgather": (4, 2048 | 1),
    "cheap_decide": (4, 128), "cheap_no_nextdir": (4, 128 | 8),
    "minb6": (4, 0, 6), "tpb128": (4, 0, 10, 128),
    "prefetch": (4, 0, 5, 256, ["-DGP_PREFETCH=1"]), "sc1st": (4, 0, 5, 256, ["-DGP_NT_STORES=2"]),
    "plainst": (4, 0, 5, 256, ["-DGP_NT_STORES=0"]), "plainld": (4, 0, 5, 256, ["-DGP_NT_LOADS=0"]),
}
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off"]


def build():
    os.makedirs(OUT, exist_ok=True)
    sort_obj = os.path.join(ROOT, "build", "obj", "gp_sort.o")
    procs = []
    for name, v in VARIANTS.items():
        npt, mask = v[0], v[1]
        minb = v[2] if len(v) > 2 else 5
        tpb = v[3] if len(v) > 3 else 256
        extra = v[4] if len(v) > 4 else []
        obj = os.path.join(OUT, f"gp_round_{name}.o")
        cmd = ["/opt/rocm/bin/hipcc", *FLAGS, f"-DGP_NPT={npt}", f"-DGP_ABLATE={mask}", f"-DGP_MINB={minb}", f"-DGP_TPB={tpb}", *extra,
               "-c", "-o", obj, os.path.join(CSRC, "gp_round.hip")]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        assert p.wait() == 0
    objdir = os.path.join(ROOT, "build", "obj")
    for name in VARIANTS:
        so = os.path.join(OUT, f"lib_{name}.so")
        objs = [os.path.join(objdir, f) for f in ("gp_api.o", "gp_kernels.o", "gp_wave.o", "gp_col.o", "gp_xchg.o",
                                                  "gp_full.o", "gp_xtile.o")]
        objs += [os.path.join(OUT, f"gp_round_{name}.o"), sort_obj]
        subprocess.check_call(["/opt/rocm/bin/hipcc", *FLAGS, "-shared", "-o", so, *objs, "-L/opt/rocm/lib", "-lrccl"])


def run(n, only=None):
    import json
    res = {}
    for name in (only or VARIANTS):
        so = os.path.join(OUT, f"lib_{name.split('@')[0]}.so")
        code = ("import sys,json; sys.path.insert(0,%r)\n"
                "from gossipprotocol_amd import Simulation\n"
                "s=Simulation(%d,%r,'push-sum',kernel_timing=True)\n"
                "P=s.population\n"
                "pre=0\nwhile s.info().active < P and pre < 300: pre += len(s.step(8))\n"
                "s.sync(); s.kernel_stats(reset=True); s.step(10); s.sync()\n"
                "ms,k,_=s.kernel_stats(); print(json.dumps(ms/k))\n") % (ROOT, n, os.environ.get("ABLATE_TOPO", "Imp3D"))
        env = dict(os.environ, GOSSIP_HIP_LIB_EXPERIMENT=so)
        if "@" in name:
            name, grid = name.split("@")
            so = os.path.join(OUT, f"lib_{name}.so")
            env.update(GOSSIP_HIP_LIB_EXPERIMENT=so, GP_GRID=grid)
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode:
            print(name, "FAILED", out.stderr[-500:], flush=True)
            sys.exit(1)
        res[name] = float(out.stdout.strip().splitlines()[-1])
        print(f"{name:14s} {res[name]:8.2f} ms/round", flush=True)
    for grid in ((8192, 16384, 32768) if not only and os.environ.get("ABLATE_GRIDS") else ()):
        so = os.path.join(OUT, "lib_base_npt4.so")
        code = ("import sys,json; sys.path.insert(0,%r)\n"
                "from gossipprotocol_amd import Simulation\n"
                "s=Simulation(%d,'Imp3D','push-sum',kernel_timing=True)\n"
                "P=s.population\n"
                "pre=0\nwhile s.info().active < P and pre < 300: pre += len(s.step(8))\n"
                "s.sync(); s.kernel_stats(reset=True); s.step(10); s.sync()\n"
                "ms,k,_=s.kernel_stats(); print(json.dumps(ms/k))\n") % (ROOT, n)
        env = dict(os.environ, GOSSIP_HIP_LIB_EXPERIMENT=so, GP_GRID=str(grid))
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode:
            print("grid", grid, "FAILED", out.stderr[-500:], flush=True)
            sys.exit(1)
        print(f"base grid={grid:<9d} {float(out.stdout.strip().splitlines()[-1]):8.2f} ms/round", flush=True)
    return res


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 10**9, sys.argv[3].split(",") if len(sys.argv) > 3 else None)
