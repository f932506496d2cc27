"""The records exchange issues the same all-reduce sequence on every rank (CPU).

tests/c/xsched_sim.cpp links the real native driver (tk_solver_run) and the exchange
schedule (csrc/tk_xsched.h) against a stand-in of tk_abi.cpp's exchange bookkeeping and
logs each rank's all-reduces (first slot, last slot, element count).  A job mixes rank
kinds whose local state differs -- one-sweep kernels that write a step's record one launch
later, two-sweep kernels, a rank holding no factor -- and different thread counts, issue
depths and TKHIP_XCH_GROUP values.  Every rank must log the same sequence;
without the agreement (tk_decomp_agree, the create preflight) they must not.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c", "xsched_sim.cpp")
CSRC = os.path.join(ROOT, "tensorkrylov.jl_amd", "csrc")
OUT = os.path.join(ROOT, "tests", "c", "_build", "xsched_sim")


@pytest.fixture(scope="module")
def sim():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.run(["g++", "-O1", "-std=c++17", "-mavx2", "-mfma", "-pthread", "-Wall", "-Wno-unknown-pragmas",
                    "-I", os.path.join(ROOT, "include"), SRC, os.path.join(CSRC, "tk_solver.cpp"),
                    os.path.join(CSRC, "tk_host.cpp"), "-o", OUT], check=True)
    return OUT


def _run(sim, local):
    env = dict(os.environ, XSCHED_SIM_LOCAL="1" if local else "0")
    p = subprocess.run([sim], capture_output=True, text=True, env=env, timeout=120)
    jobs = [l for l in p.stdout.splitlines() if l.startswith("JOB ")]
    return p, jobs


def test_every_rank_issues_the_same_allreduces(sim):
    p, jobs = _run(sim, local=False)
    assert p.returncode == 0, p.stdout + p.stderr
    assert len(jobs) == 11
    for line in jobs:
        assert "identical=1" in line, line
    # the default group of 4 batches the step slots once the issue depth covers a group
    first = jobs[0]
    assert "[2,5]x3520" in first and "[46,49]x3520" in first, first
    # converged job: the flush slot (kmax + 1) goes out once, after every issued step's slot
    conv = [l for l in jobs if l.startswith("JOB converged")][0]
    assert conv.split("first=")[1].split()[-5] == "[51,51]x880", conv


def test_without_agreement_ranks_diverge(sim):
    """Negative control: per-rank worker counts / group sizes give different sequences
    (the hang or record mix-up the agreement prevents)."""
    p, jobs = _run(sim, local=True)
    assert p.returncode == 1
    assert any("identical=0" in l for l in jobs)


def test_evaluation_split_over_ranks(sim):
    """tk_solver_share: ranks running concurrently, each evaluating the
    iterations k = rank (mod nranks) and reading the others' results from the real
    shared-memory mailbox, issue the same all-reduces and end at the same iteration with the
    same outcome and residual (the log's last entries); a rank that converges on another
    rank's iteration still returns its y (tk_solver_solution).  With one rank lacking a
    results source the run's agreement turns the split off everywhere.  No file is left in
    /dev/shm."""
    before = set(os.listdir("/dev/shm")) if os.path.isdir("/dev/shm") else set()
    p, jobs = _run(sim, local=False)
    assert p.returncode == 0, p.stdout + p.stderr
    split = [l for l in jobs if l.startswith("JOB split")]
    assert len(split) == 4
    for line in split:
        assert "identical=1" in line, line
    conv = [l for l in split if l.startswith("JOB split-converged")][0]
    assert "outcome=1" in conv
    after = set(os.listdir("/dev/shm")) if os.path.isdir("/dev/shm") else set()
    assert not [f for f in after - before if f.startswith("tkhip_ev_")]
