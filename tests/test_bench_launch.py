"""bench.py --gpus N without a launcher: the process starts
torch.distributed.run as a CHILD -- N ranks, 127.0.0.1 rendezvous, the same arguments --
before anything in it loads the HIP runtime or libtkhip, and exits with the child's status.
The torchrun form (`python -m torch.distributed.run ... bench.py --gpus N`) stays valid:
WORLD_SIZE set means "I am a rank", so no second launch happens."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def test_launcher_argv():
    sys.path.insert(0, ROOT)
    import bench
    argv = bench.launcher_argv(4, ["--gpus", "4", "--steps", "7", "--config", "C4"], 29555)
    assert argv[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in argv
    assert argv[argv.index("--nproc-per-node") + 1] == "4"
    assert argv[argv.index("--master-addr") + 1] == "127.0.0.1"
    assert argv[argv.index("--master-port") + 1] == "29555"
    i = argv.index(BENCH)
    assert argv[i + 1:] == ["--gpus", "4", "--steps", "7", "--config", "C4"]


def test_parent_launches_child_without_touching_the_gpu():
    """The parent's only action is the child launch (stubbed here): afterwards neither the HIP
    runtime nor libtkhip is mapped into it, tkamd was never imported, and its exit status is
    the child's."""
    code = r'''
import json, os, subprocess, sys
sys.path.insert(0, %r)
os.environ.pop("WORLD_SIZE", None)
sys.argv = ["bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1"]
import bench
calls = []
class FakeChild:
    def __init__(self, argv, env=None):
        calls.append((argv, env.get("MASTER_ADDR")))
    def wait(self):
        return 5
subprocess.Popen = FakeChild
rc = bench.main()
maps = open("/proc/self/maps").read()
print(json.dumps({"rc": rc, "argv": calls[0][0], "addr": calls[0][1], "ncalls": len(calls),
                  "hip": "libamdhip64" in maps, "tk": "libtkhip" in maps,
                  "tkamd": "tkamd" in sys.modules}))
''' % ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["rc"] == 5 and out["ncalls"] == 1
    assert out["argv"][out["argv"].index("--nproc-per-node") + 1] == "2"
    assert out["argv"][-6:] == ["--gpus", "2", "--steps", "3", "--warmup", "1"]
    assert out["addr"] == "127.0.0.1"
    assert not out["hip"] and not out["tk"] and not out["tkamd"]


def test_self_launch_runs_ranks_and_returns_their_status():
    """The real child on this GPU-less container: torch.distributed.run starts 2 ranks of
    bench.py (WORLD_SIZE=2 in their environment, so neither relaunches); each fails at its
    context (no gfx950 device) with its diagnosis, and the parent exits non-zero."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline", "--no-end-to-end"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode != 0
    err = p.stderr
    # (torchrun stops the other rank once one has failed: at least one diagnosis is printed)
    assert "bench.py rank 0" in err or "bench.py rank 1" in err, err[-3000:]
    assert "no HIP device" in err or "gfx950" in err
