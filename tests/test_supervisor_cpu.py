"""The bench's fail-safe launcher (utils/supervisor.py, bench.py main) on CPU.

VERDICT r2 item 1: ``bench.py --gpus N`` must start N ranks itself, a failing or hanging
rank must move every rank to the next fallback level (or fail the run), and the launcher /
flag disagreement must be an error.  The GPU worker is replaced by tests/sup_worker.py.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from network_distributed_pytorch_amd.utils import supervisor as sup  # noqa: E402
from network_distributed_pytorch_amd.utils.launcher import find_free_port  # noqa: E402

WORKER = [sys.executable, "-u", os.path.join(ROOT, "tests", "sup_worker.py")]


@pytest.fixture
def clean_env(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_USE_AGENT_STORE",
              sup.ROLE_ENV, sup.DIR_ENV, sup.LEVEL_ENV):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    return monkeypatch


def test_local_success_level0(clean_env):
    clean_env.setenv("SUP_TEST_DIST", "1")
    att = sup.supervise_local(WORKER, world=2, levels=3)
    assert len(att) == 1 and att[0].ok and att[0].level == 0
    rec = json.loads(att[0].result)
    assert rec["world"] == 2 and rec["level"] == 0


@pytest.mark.parametrize("action", ["fail", "crash", "hang"])
def test_local_failure_falls_back_on_every_rank(clean_env, action):
    clean_env.setenv("SUP_TEST_DIST", "1")
    clean_env.setenv("SUP_TEST_MODE", f"0:1:{action}")
    att = sup.supervise_local(WORKER, world=2, levels=3)
    assert [a.ok for a in att] == [False, True]
    assert 1 in att[0].errors
    if action == "fail":
        assert "boom at level 0" in att[0].errors[1]
    if action == "hang":
        assert "stalled in phase 'hang'" in att[0].errors[1]
    rec = json.loads(att[1].result)
    assert rec["level"] == 1 and rec["world"] == 2
    line = json.loads(sup.attach_attempts(att[1].result, att))
    assert line["supervisor"]["level"] == 1 and line["supervisor"]["failed"][0]["level"] == 0


def test_local_all_levels_fail_exit_code(clean_env, capsys):
    clean_env.setenv("SUP_TEST_MODE", "0:*:fail,1:0:fail")
    code = sup.run_supervised(WORKER, world=2, levels=2)
    assert code == 1
    assert capsys.readouterr().out == ""  # no number is printed for an unverified run


def test_teardown_crash_after_done_still_counts(clean_env):
    clean_env.setenv("SUP_TEST_MODE", "0:1:late")
    att = sup.supervise_local(WORKER, world=2, levels=2)
    assert att[0].ok and "teardown" in att[0].errors[1]


def test_first_level(clean_env):
    att = sup.supervise_local(WORKER, world=1, levels=3, first_level=2)
    assert att[0].level == 2 and json.loads(att[0].result)["level"] == 2


def _torchrun(tmp_path, nproc, mode, extra_env=None):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update({"SUP_TEST_MODE": mode, "SUP_TEST_DIST": "1", "OMP_NUM_THREADS": "1",
                 "PYTHONPATH": ROOT + os.pathsep + env.get("PYTHONPATH", "")})
    env.update(extra_env or {})
    driver = tmp_path / "drv.py"
    driver.write_text(
        "import os, sys\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "from network_distributed_pytorch_amd.utils import supervisor as sup\n"
        f"sys.exit(sup.run_supervised({WORKER!r}, world=int(os.environ['WORLD_SIZE']), levels=3))\n")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(find_free_port()), str(driver)]
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)


def test_torchrun_mode_agrees_on_fallback(tmp_path):
    p = _torchrun(tmp_path, 2, "0:1:fail")
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["level"] == 1 and rec["world"] == 2
    assert rec["supervisor"]["failed"][0]["level"] == 0
    assert "boom" in rec["supervisor"]["failed"][0]["errors"]["1"]


def test_torchrun_mode_peer_hang_kills_healthy_rank(tmp_path):
    # rank 0 hangs at level 0: rank 1 (blocked in the gloo rendezvous / all_reduce) must be
    # killed through the shared fail key, and both ranks must succeed at level 1
    p = _torchrun(tmp_path, 2, "0:0:hang")
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["level"] == 1


def test_bench_world_mismatch(clean_env):
    clean_env.setenv("WORLD_SIZE", "2")
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.resolve_world(bench.parse(["--gpus", "4"]))
    assert bench.resolve_world(bench.parse([])) == 2
    clean_env.delenv("WORLD_SIZE")
    assert bench.resolve_world(bench.parse(["--gpus", "8"])) == 8
    assert bench.resolve_world(bench.parse([])) == 1
    assert len(bench.fallbacks(8)) == 4 and bench.fallbacks(1)[0] == {}
