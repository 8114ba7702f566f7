"""Akka reference timing wrapper (§8(d) "CPU beside it" (2)).

    python tools/akka_timing.py [--nodes 1000] [--topology line] [--algorithm gossip]
                                [--reference /root/reference] [--timeout 600] [--cores N]

Runs the original F#/Akka.NET program the way its README.md:1 says (`dotnet run
<num_nodes> <topology> <algorithm>`), from a scratch copy of `Project2/` (the
reference tree is read-only), with
  * stdin redirected from /dev/null: the program ends in `Console.ReadKey()`
    (Program.fs:282) on the paths that do not call `Environment.Exit`;
  * a wall-clock timeout: the reference can live-lock;
  * optional core pinning (`taskset -c 0..N-1`) so the reported core count is exact.
It parses `Convergence Time: %f ms` (Program.fs:55) and prints one JSON line with
the core count — a reported baseline only, never a parity check (the reference is
asynchronous and clock-seeded).  Where no .NET SDK is installed (this image and the
GPU boxes) it reports `"available": false` with the reason instead.
"""
import argparse
import json
import os
import re
import shutil
import signal
import subprocess
import tempfile
import time

CONV_RE = re.compile(r"Convergence Time:\s*([0-9.eE+-]+)\s*ms")


def parse_convergence_ms(stdout: str):
    """The reference's only result line (Program.fs:55), or None."""
    m = CONV_RE.search(stdout)
    return float(m.group(1)) if m else None


def run_reference(nodes, topology, algorithm, reference="/root/reference", timeout=600, cores=0,
                  dotnet=None):
    dotnet = dotnet or shutil.which("dotnet")
    cfg = {"nodes": nodes, "topology": topology, "algorithm": algorithm}
    if not dotnet:
        return {"available": False, "reason": "no dotnet (no .NET SDK on this host)", **cfg}
    proj = os.path.join(reference, "Project2")
    if not os.path.isdir(proj):
        return {"available": False, "reason": f"reference project not found at {proj}", **cfg}
    ncpu = os.cpu_count() or 1
    with tempfile.TemporaryDirectory(prefix="akka_ref_") as tmp:
        work = os.path.join(tmp, "Project2")
        shutil.copytree(proj, work, ignore=shutil.ignore_patterns("bin", "obj"))
        # build first (restore + compile are not part of the timed run; with no
        # package source the restore fails, reported as unavailable with the reason)
        rc, out, err, _ = _run_group([dotnet, "build", "-c", "Release"], work, timeout)
        if rc != 0:
            why = "timeout" if rc is None else f"exit {rc}"
            return {"available": False, "reason": f"dotnet build failed ({why}): {(out + err)[-300:]}", **cfg}
        cmd = [dotnet, "run", "--no-build", "-c", "Release", "--", str(nodes), topology, algorithm]
        used = ncpu  # cores the run may use: pinned only when taskset is really applied
        if cores > 0 and shutil.which("taskset"):
            used = min(cores, ncpu)
            cmd = ["taskset", "-c", f"0-{used - 1}"] + cmd
        t0 = time.perf_counter()
        rc, out, _, timed_out = _run_group(cmd, work, timeout)
        wall = time.perf_counter() - t0
    if timed_out:
        return {"available": True, "converged": False, "reason": f"timeout after {timeout} s", "cores": used, **cfg}
    ms = parse_convergence_ms(out)
    return {"available": True, "converged": ms is not None, "convergence_ms": ms, "wall_s": wall,
            "exit_code": rc, "cores": used, **cfg}


def _run_group(cmd, cwd, timeout):
    """Run cmd in its own session; on timeout kill the whole process group (the
    app process `dotnet run` spawns would otherwise outlive it, live-locked on the
    pinned cores).  Returns (returncode or None, stdout, stderr, timed_out)."""
    p = subprocess.Popen(cmd, cwd=cwd, stdin=subprocess.DEVNULL, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True, start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
        return p.returncode, out, err, False
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        return None, out or "", err or "", True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1000)
    ap.add_argument("--topology", default="line")
    ap.add_argument("--algorithm", default="gossip")
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--timeout", type=int, default=600)
    ap.add_argument("--cores", type=int, default=0)
    a = ap.parse_args()
    print(json.dumps(run_reference(a.nodes, a.topology, a.algorithm, a.reference, a.timeout, a.cores)), flush=True)


if __name__ == "__main__":
    main()
