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
