"""bench.py's multi-GPU launch contract, on the CPU.

`python bench.py --gpus N` outside torchrun must start N ranks itself
(torch.distributed.run, rendezvous on 127.0.0.1) without the launcher
process ever loading the HIP library, and print exactly one JSON line; a
WORLD_SIZE that disagrees with --gpus must end the run non-zero.  The hidden
--launch-probe mode replaces the GPU work by a gloo rendezvous in which each
rank reports RANK / LOCAL_RANK / WORLD_SIZE."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(HPXHIP_COLLECTIVE_TIMEOUT_S="60", **kw)
    return env


@pytest.mark.parametrize("n", [2, 4])
def test_gpus_n_starts_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-probe"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]  # gloo logs its own lines
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["launch_probe"] and d["n_gpus"] == n and d["ranks"] == n
    envs = d["rank_env"]
    assert [e["RANK"] for e in envs] == list(range(n))
    assert sorted(e["LOCAL_RANK"] for e in envs) == list(range(n))
    assert all(e["WORLD_SIZE"] == n for e in envs)
    assert len({e["pid"] for e in envs}) == n          # one process per rank
    assert not any(e["hip_library_loaded"] for e in envs)


def test_single_gpu_stays_in_process():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--launch-probe"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip())
    assert d["ranks"] == 1 and d["rank_env"][0]["pid"] != os.getpid()


def test_world_size_mismatch_is_an_error():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--launch-probe"], cwd=ROOT,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and r.stdout.strip() == ""


def test_launcher_never_imports_the_library():
    """The launcher path returns before `import hpx_amd`: run main() in a
    child with the library import poisoned and a fake torch.distributed.run
    that only records its argv."""
    code = (
        "import sys, subprocess, json\n"
        "sys.modules['hpx_amd'] = None\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "calls = []\n"
        "subprocess.call = lambda cmd, env=None: calls.append(cmd) or 0\n"
        "import bench\n"
        "try:\n"
        "    bench.main(['--gpus', '8', '--steps', '3'])\n"
        "except SystemExit as e:\n"
        "    assert e.code == 0, e.code\n"
        "cmd = calls[0]\n"
        "assert cmd[1:3] == ['-m', 'torch.distributed.run'] and '--nproc-per-node=8' in cmd, cmd\n"
        "assert '--master-addr=127.0.0.1' in cmd and cmd[-3:] == ['--gpus', '8', '--steps', '3'][-3:], cmd\n"
        "assert 'torch' not in sys.modules\n"
        "print('ok')\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-3000:]
