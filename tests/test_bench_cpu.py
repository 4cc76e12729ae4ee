"""bench.py's multi-rank contract on CPU (no GPU touched): ``--gpus N``
without a torch.distributed launcher starts N ranks as child processes and
relays rank 0's JSON line; WORLD_SIZE != --gpus is an error."""
import importlib.util
import os
import subprocess
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_check_world(monkeypatch):
    b = _bench()
    args = types.SimpleNamespace(gpus=1)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert b.check_world(args) is None
    args.gpus = 4
    assert b.check_world(args) == ("launch", 4)
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert b.check_world(args) is None
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert b.check_world(args)[0] == "error"


def test_relay_picks_the_result_line():
    b = _bench()
    out = "RCCL version 2.x\n{\"not\": 1}\nnoise {\n{\"metric\": \"m\", \"value\": 3, \"n_gpus\": 2}\ntrailer\n"
    assert b.relay_json(out) == "{\"metric\": \"m\", \"value\": 3, \"n_gpus\": 2}"
    assert b.relay_json("nothing here") is None


def test_launch_ranks_runs_torch_distributed_and_relays(capsys):
    b = _bench()
    seen = {}

    def runner(cmd, stdout=None, env=None, text=None):
        seen["cmd"], seen["env"] = cmd, env
        return types.SimpleNamespace(returncode=0, stdout="banner\n{\"metric\": \"x\", \"n_gpus\": 2}\n")

    args = types.SimpleNamespace(gpus=2)
    rc = b.launch_ranks(args, ["--gpus", "2", "--steps", "3"], runner=runner)
    assert rc == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-4:] == ["--gpus", "2", "--steps", "3"] and cmd[-5].endswith("bench.py")
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert capsys.readouterr().out.strip() == "{\"metric\": \"x\", \"n_gpus\": 2}"


def test_launch_ranks_failure_is_nonzero():
    b = _bench()
    runner = lambda cmd, **kw: types.SimpleNamespace(returncode=3, stdout="boom")  # noqa: E731
    assert b.launch_ranks(types.SimpleNamespace(gpus=2), [], runner=runner) == 3
    runner = lambda cmd, **kw: types.SimpleNamespace(returncode=0, stdout="no json")  # noqa: E731
    assert b.launch_ranks(types.SimpleNamespace(gpus=2), [], runner=runner) == 1


def test_world_size_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_per_rank_batch_splits_the_global_c4_c5_batch():
    """BASELINE configs[3] (C4: batch 4096 across 8×MI355X, SURVEY §8e: 512
    sessions per rank) and configs[4] (C5: batch 8192) are global batches:
    their ranks split them; C2 / C3 keep 4096 per GPU (weak scaling)."""
    b = _bench()
    assert [b.per_rank_batch("c4", 4096, w) for w in (1, 2, 4, 8)] == [4096, 2048, 1024, 512]
    assert [b.per_rank_batch("c5", 8192, w) for w in (1, 2, 4, 8)] == [8192, 4096, 2048, 1024]
    assert [b.per_rank_batch("c2", 4096, w) for w in (1, 2, 8)] == [4096] * 3
    with pytest.raises(SystemExit):
        b.per_rank_batch("c4", 4096, 3)


def test_host_threads_reports_the_usable_cpus():
    b = _bench()
    n, how = b.host_threads()
    assert 1 <= n <= how["affinity_cpus"]
    if how["cgroup_cpu_quota"]:
        assert n <= how["cgroup_cpu_quota"]


def test_loss_parity_bars():
    """The C2 line's loss_parity (GPU trainer vs the oracle on the same first
    batches): the bars of tests/test_gpu_supervised.py."""
    import torch
    b = _bench()
    sd = {"w": torch.zeros(1000), "b": torch.zeros(10)}
    near = {"w": torch.zeros(1000), "b": torch.full((10,), 5e-5)}
    ok = b.loss_parity([9.1, 9.2], [9.10005, 9.2], sd, near, 0.01, 4096)
    assert ok["pass"] and ok["steps"] == 2 and ok["max_abs_dloss"] < 1e-4
    assert ok["params"]["b"]["max_abs"] == pytest.approx(5e-5) and ok["params"]["b"]["frac_gt_1e-4"] == 0
    assert not b.loss_parity([9.1], [9.1003], sd, near, 0.01, 4096)["pass"]
    flip = {"w": torch.zeros(1000), "b": torch.zeros(10)}
    flip["w"][:2] = 0.02   # two sign-like Adam flips of 2·lr in 1000 elements: 0.2 % > 0.1 %
    assert not b.loss_parity([9.1], [9.1], sd, flip, 0.01, 4096)["pass"]


def test_pmc_traffic_needs_the_measured_sources(tmp_path, monkeypatch):
    """A PMC traffic entry counts only while its source hash matches the
    current kernel sources (bench.py kernel_src_hash)."""
    import json
    b = _bench()
    h = b.kernel_src_hash("head")
    assert len(h) == 16 and h == b.kernel_src_hash("head") and h != b.kernel_src_hash("gather+sampled_fwd")
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_traffic.json").write_text(json.dumps({
        "head_fwd:f32x6d3:zs": {"bytes": 123, "src": h, "file": "x"},
        "head_dw_adam:f32x6d3:zs": {"bytes": 456, "src": "0" * 16, "file": "y"},
        "old": 789}))
    csrc = tmp_path / "ikea-recommender-system_amd" / "csrc"
    csrc.mkdir(parents=True)
    for f in b.KERNEL_SRC["head"]:
        (csrc / f).write_bytes(open(os.path.join(ROOT, "ikea-recommender-system_amd", "csrc", f), "rb").read())
    monkeypatch.setattr(b, "HERE", str(tmp_path))
    assert b.pmc_traffic("head_fwd:f32x6d3:zs", "head") == 123
    assert b.pmc_traffic("head_dw_adam:f32x6d3:zs", "head") is None   # measured on other sources
    assert b.pmc_traffic("old", "head") is None                       # unversioned entry
    assert b.pmc_traffic("missing", "head") is None
