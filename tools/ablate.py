"""Ablation study of the round kernel (experiment tool, not part of the product).

    python tools/ablate.py build            # CPU: compile variants into build/ablate/
    python tools/ablate.py run [n]           # GPU: time each variant (steady state from round 0)

Each variant compiles gp_kernels.hip / gp_api.hip with -DGP_ABLATE=<mask>
(switch meanings at the top of gp_kernels.hip); results are wrong by design,
only the time per round matters.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gossipprotocol_amd", "csrc")
OUT = os.path.join(ROOT, "build", "ablate")
VARIANTS = {
    "base": 1, "no_inlist": 1 | 2, "no_rgather": 1 | 4, "no_lattice": 1 | 8, "no_nextdir": 1 | 16,
    "no_ratio": 1 | 32, "lattice_only": 1 | 2 | 16 | 32, "stream_only": 1 | 2 | 8 | 16 | 32,
}
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off"]


def build():
    os.makedirs(OUT, exist_ok=True)
    sort_obj = os.path.join(ROOT, "build", "obj", "gp_sort.o")
    procs = []
    for name, mask in VARIANTS.items():
        for src in ("gp_api", "gp_kernels"):
            obj = os.path.join(OUT, f"{src}_{name}.o")
            cmd = ["/opt/rocm/bin/hipcc", *FLAGS, f"-DGP_ABLATE={mask}", "-c", "-o", obj,
                   os.path.join(CSRC, src + ".hip")]
            procs.append(subprocess.Popen(cmd))
    for p in procs:
        assert p.wait() == 0
    for name in VARIANTS:
        so = os.path.join(OUT, f"lib_{name}.so")
        objs = [os.path.join(OUT, f"{src}_{name}.o") for src in ("gp_api", "gp_kernels")] + [sort_obj]
        subprocess.check_call(["/opt/rocm/bin/hipcc", *FLAGS, "-shared", "-o", so, *objs])


def run(n):
    import json
    res = {}
    for name in VARIANTS:
        so = os.path.join(OUT, f"lib_{name}.so")
        code = ("import sys,json; sys.path.insert(0,%r)\n"
                "from gossipprotocol_amd import Simulation\n"
                "s=Simulation(%d,'Imp3D','push-sum',kernel_timing=True)\n"
                "s.step(3); s.sync(); s.kernel_stats(reset=True); s.step(10); s.sync()\n"
                "ms,k,_=s.kernel_stats(); print(json.dumps(ms/k))\n") % (ROOT, n)
        env = dict(os.environ, GOSSIP_HIP_LIB_EXPERIMENT=so)
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode:
            print(name, "FAILED", out.stderr[-500:], flush=True)
            break
        res[name] = float(out.stdout.strip().splitlines()[-1])
        print(f"{name:14s} {res[name]:8.2f} ms/round", flush=True)
    for grid in (1024, 4096, 16384, 65536, (n + 255) // 256):
        so = os.path.join(OUT, "lib_base.so")
        code = ("import sys,json; sys.path.insert(0,%r)\n"
                "from gossipprotocol_amd import Simulation\n"
                "s=Simulation(%d,'Imp3D','push-sum',kernel_timing=True)\n"
                "s.step(3); s.sync(); s.kernel_stats(reset=True); s.step(10); s.sync()\n"
                "ms,k,_=s.kernel_stats(); print(json.dumps(ms/k))\n") % (ROOT, n)
        env = dict(os.environ, GOSSIP_HIP_LIB_EXPERIMENT=so, GP_GRID=str(grid))
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode:
            print("grid", grid, "FAILED", out.stderr[-500:], flush=True)
            break
        print(f"base grid={grid:<9d} {float(out.stdout.strip().splitlines()[-1]):8.2f} ms/round", flush=True)
    return res


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 10**9)
