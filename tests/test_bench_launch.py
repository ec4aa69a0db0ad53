"""CPU tests of bench.py's rank launcher: `python bench.py --gpus N` starts its own N ranks
(torch.distributed.run as a child process, one process per GPU) and a rank refuses a
WORLD_SIZE that differs from --gpus.  Nothing here touches a GPU."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_launcher_argv():
    argv = bench.launcher_argv(8, ["--gpus", "8", "--steps", "5"], 29555, python="/usr/bin/python3",
                               script="/x/bench.py")
    assert argv == ["/usr/bin/python3", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                    "--master-addr", "127.0.0.1", "--master-port", "29555", "/x/bench.py",
                    "--gpus", "8", "--steps", "5"]


def test_check_world():
    assert bench.check_world(1, env={}) is False          # plain N = 1 run: this process is rank 0
    assert bench.check_world(4, env={}) is True           # N > 1 outside a launcher: spawn
    assert bench.check_world(4, env={"WORLD_SIZE": "4"}) is False   # a rank of the launcher
    assert bench.check_world(1, env={"WORLD_SIZE": "1"}) is False
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.check_world(4, env={"WORLD_SIZE": "2"})


def test_spawned_ranks_reach_rank_code(tmp_path):
    """End to end on the CPU: the parent builds the launcher command and the child
    torch.distributed.run starts 2 ranks of a stand-in script that reports its env; the
    parent's exit status is the child's."""
    probe = tmp_path / "probe.py"
    out = tmp_path / "ranks"
    out.mkdir()
    probe.write_text("import os, sys\n"
                     "open(os.path.join(%r, os.environ['RANK']), 'w').write(os.environ['WORLD_SIZE'] + ' ' + "
                     "' '.join(sys.argv[1:]))\n" % str(out))
    cmd = bench.launcher_argv(2, ["--gpus", "2"], bench._free_port(), script=str(probe))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    rc = subprocess.call(cmd, env=env, timeout=120, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    assert rc == 0
    got = sorted(os.listdir(out))
    assert got == ["0", "1"]
    for r in got:
        assert (out / r).read_text() == "2 --gpus 2"
