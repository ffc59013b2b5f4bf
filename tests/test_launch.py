"""`bench.py --gpus N` / `bench_loop.py --gpus N` start N rank processes
(dgen_amd/launch.py) when no torch.distributed.run environment is present,
and refuse a world size that differs from --gpus.  CPU only: the launched
children here are a tiny gloo script, never the GPU benchmark."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

from dgen_amd import launch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plan_has_one_env_per_rank():
    plan = launch.launch_plan(4, "bench.py", ["--gpus", "4", "--steps", "3"], port=29999, base={"A": "1"})
    assert len(plan) == 4
    for r, (cmd, env) in enumerate(plan):
        assert cmd[0] == sys.executable and cmd[-4:] == ["--gpus", "4", "--steps", "3"]
        assert os.path.basename(cmd[2]) == "bench.py"
        assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"], env["LOCAL_WORLD_SIZE"]) == (str(r), str(r), "4", "4")
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29999"
        assert env["A"] == "1" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_world_mismatch_is_refused(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert launch.check_world(8) == 2
    assert launch.maybe_launch(8, "bench.py", []) == 2
    assert launch.maybe_launch(2, "bench.py", []) is None      # a torchrun rank: runs itself
    monkeypatch.delenv("WORLD_SIZE")
    assert launch.maybe_launch(1, "bench.py", []) is None      # the single-GPU run


def _child_script(tmp_path):
    p = tmp_path / "child.py"
    p.write_text(textwrap.dedent(f"""
        import json, os, sys
        sys.path.insert(0, {REPO!r})
        from dgen_amd.launch import maybe_launch
        gpus = int(sys.argv[1])
        st = maybe_launch(gpus, __file__, sys.argv[1:])
        if st is not None:
            sys.exit(st)
        import torch, torch.distributed as dist
        dist.init_process_group("gloo")
        t = torch.tensor([float(dist.get_rank() + 1)])
        dist.all_reduce(t)
        if os.environ.get("FAIL_RANK") == os.environ["RANK"]:
            sys.exit(3)
        if dist.get_rank() == 0:
            print(json.dumps({{"n_gpus": dist.get_world_size(), "sum": float(t.item())}}), flush=True)
        dist.destroy_process_group()
    """))
    return str(p)


def test_parent_launches_n_ranks_without_touching_torch(tmp_path):
    script = _child_script(tmp_path)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, script, "3"], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines == [{"n_gpus": 3, "sum": 6.0}]                # one line, from rank 0
    # the parent itself never imports torch: checked in-process
    code = ("import sys; sys.path.insert(0, %r); import dgen_amd.launch; "
            "print('torch' in sys.modules)" % REPO)
    assert subprocess.run([sys.executable, "-c", code], capture_output=True, text=True).stdout.strip() == "False"


def test_failing_rank_fails_the_launch(tmp_path):
    script = _child_script(tmp_path)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["FAIL_RANK"] = "1"
    r = subprocess.run([sys.executable, script, "2"], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])


@pytest.mark.parametrize("script", ["bench.py", "bench_loop.py"])
def test_bench_scripts_refuse_world_mismatch(script):
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, script), "--gpus", "8"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr, r.stderr[-2000:]
