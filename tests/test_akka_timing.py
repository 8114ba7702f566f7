"""Akka reference timing wrapper (tools/akka_timing.py): output parsing and the
"no .NET" report.  The reference itself is never run here (no dotnet in the image)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import akka_timing as at  # noqa: E402


def test_parse_convergence_line():
    out = "Gossip Starts\nConvergence Time: 1234.567800 ms\n"  # Program.fs:198, 55
    assert at.parse_convergence_ms(out) == 1234.5678
    assert at.parse_convergence_ms("option invalid\n") is None  # Program.fs:207


def test_unavailable_without_dotnet(monkeypatch):
    monkeypatch.setattr(at.shutil, "which", lambda name: None)
    r = at.run_reference(1000, "line", "gossip")
    assert r["available"] is False and "dotnet" in r["reason"]
    assert (r["nodes"], r["topology"], r["algorithm"]) == (1000, "line", "gossip")


def test_missing_reference_project(tmp_path):
    r = at.run_reference(10, "full", "push-sum", reference=str(tmp_path), dotnet="/bin/true")
    assert r["available"] is False and "not found" in r["reason"]


def _fake_reference(tmp_path):
    proj = tmp_path / "Project2"
    proj.mkdir()
    (proj / "Program.fs").write_text("// stand-in project directory (never compiled)\n")
    return str(tmp_path)


def _fake_dotnet(tmp_path, body):
    exe = tmp_path / "dotnet"
    exe.write_text("#!/bin/bash\n" + body)
    exe.chmod(0o755)
    return str(exe)


def test_build_failure_reported_unavailable(tmp_path):
    dn = _fake_dotnet(tmp_path, 'if [ "$1" = build ]; then echo "restore failed: no network"; exit 1; fi\n')
    r = at.run_reference(10, "line", "gossip", reference=_fake_reference(tmp_path), dotnet=dn)
    assert r["available"] is False and "build failed" in r["reason"] and "restore failed" in r["reason"]


def test_timed_run_parses_and_kills_group_on_timeout(tmp_path):
    dn = _fake_dotnet(tmp_path, 'if [ "$1" = build ]; then exit 0; fi\n'
                      'if [ "$8" = slow ]; then sleep 30 & wait; fi\n'
                      'echo "Convergence Time: 12.5 ms"\n')
    ref = _fake_reference(tmp_path)
    r = at.run_reference(10, "line", "gossip", reference=ref, dotnet=dn)
    assert r["available"] and r["converged"] and r["convergence_ms"] == 12.5
    r = at.run_reference(10, "line", "slow", reference=ref, dotnet=dn, timeout=1)
    assert r["available"] and r["converged"] is False and "timeout" in r["reason"]
