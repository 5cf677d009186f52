"""bench.py's rank launcher (the driver runs `python bench.py --gpus N`, and also
`torch.distributed.run ... bench.py --gpus N`): N > 1 without a launcher starts N child ranks,
a mismatch with WORLD_SIZE is refused, too few GPUs is an error naming the count.  CPU only."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], env=env, capture_output=True, text=True, timeout=timeout,
                          cwd=ROOT)


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_dry_run_spawns_two_ranks():
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr
    d = _json_line(r.stdout)
    assert d["dry_run"] and d["world_size"] == 2
    assert sorted(x["rank"] for x in d["ranks"]) == [0, 1]
    assert sorted(x["local_rank"] for x in d["ranks"]) == [0, 1]
    assert all(x["world_size"] == 2 for x in d["ranks"])


def test_point_count_reaches_the_ranks():
    """--n is an ambiguous prefix of the launcher's own options (its parser reads the script's tokens
    too): the ranks still receive it."""
    for args in (["--n", "20000"], ["--n=20000"], ["--points", "20000"]):
        r = _run(["--gpus", "2", "--dry-run", *args])
        assert r.returncode == 0, r.stderr
        assert _json_line(r.stdout)["points"] == 20000


def test_dry_run_one_rank_needs_no_launcher():
    r = _run(["--gpus", "1", "--dry-run"])
    assert r.returncode == 0, r.stderr
    d = _json_line(r.stdout)
    assert d["world_size"] == 1 and d["ranks"] == [{"rank": 0, "local_rank": 0, "world_size": 1}]


def test_too_few_gpus_is_an_error_naming_the_count():
    import torch
    have = torch.cuda.device_count()
    want = have + 1
    if want < 2:
        want = 2
    r = _run(["--gpus", str(want), "--steps", "1"])
    assert r.returncode != 0
    assert f"{have} GPU(s) are visible" in r.stderr and f"--gpus {want}" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")], "no bench line on a refused run"


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "3", "--dry-run"], env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


@pytest.mark.parametrize("bad", ["0", "-1"])
def test_gpus_must_be_positive(bad):
    r = _run(["--gpus", bad, "--dry-run"])
    assert r.returncode != 0


def test_traffic_comes_only_from_a_profile_of_the_same_command():
    """roofline.traffic is read from the committed PMC summary whose key (workload, steps, warmup) is the
    line's own; another command's bytes are refused with the reason."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    wl = "3d_room_1000k_1000k_k20"
    by, f, per_pass, note = b.measured_traffic(wl, 20, 5)   # the driver's command: profiled
    assert by and by > 48e6 and f.endswith("pmc_traffic.json") and "--steps 20 --warmup 5" in note
    d = json.load(open(os.path.join(ROOT, f)))
    assert (d["workload"], d["steps"], d["warmup"], d["launches"]) == (wl, 20, 5, 205)
    assert len(per_pass["bytes_by_pass"]) == 20
    by, f, per_pass, note = b.measured_traffic(wl, 30, 5)   # not profiled: no bytes, and why
    assert by is None and f is None and "no PMC profile of this command (steps 30, warmup 5)" in note
    assert b.measured_traffic("2d_segments_1000k", 20, 5)[0] is None


class _FakeEngine:
    """The exchange surface of gicp.Engine, no GPU: peer_init fails on the ranks in `fail_on`."""

    def __init__(self, rank, world, fail_on=(), export_fail_on=()):
        self.rank, self.world, self.kind = rank, world, "none"
        self.fail_on, self.export_fail_on = set(fail_on), set(export_fail_on)
        self.calls = []

    def peer_export(self):
        self.calls.append("export")
        if self.rank in self.export_fail_on:
            raise RuntimeError("export failed (fake)")
        return bytes([self.rank]) * 72

    def peer_init(self, n, r, handles, timeout=10.0):
        self.calls.append("peer_init")
        assert len(handles) == n and all(len(h) == 72 for h in handles)
        if r in self.fail_on:
            raise RuntimeError("probe failed (fake)")
        self.kind = "peer"

    def peer_close(self):
        self.calls.append("peer_close")
        self.kind = "none"

    def comm_init(self, n, r, uid):
        self.calls.append("comm_init")
        assert uid == b"uid" * 4
        self.kind = "rccl"

    def comm_ranks(self):
        return (self.world if self.kind != "none" else 1), self.rank, self.kind


def _exchange_rank(rank, world, port, d, exchange, fail_on, export_fail_on, share_gpu):
    import json as js
    import torch.distributed as dist
    sys.path[:0] = [ROOT, os.path.join(ROOT, "generalized-icp_amd")]
    import bench
    from gicp import distributed as gd

    class _E:   # gd.init_comm's unique id (the real one asks RCCL)
        @staticmethod
        def comm_unique_id():
            return b"uid" * 4
    gd.Engine = _E
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _FakeEngine(rank, world, fail_on, export_fail_on)
    try:
        note, n, kind = bench.setup_exchange(eng, gd, rank, world, exchange, share_gpu)
        out = {"note": note, "n": n, "kind": kind, "calls": eng.calls}
    except SystemExit as e:
        out = {"exit": str(e), "calls": eng.calls}
    with open(os.path.join(d, f"x{rank}.json"), "w") as f:
        js.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case", ["all_ok", "rank1_probe_fails", "rank0_export_fails", "rccl_asked", "shared_gpu_fails"])
def test_bench_exchange_decision_is_agreed_by_every_rank(tmp_path, case):
    """bench.py's exchange set-up (setup_exchange) on two gloo ranks with a fake engine: when the peer
    exchange fails on ANY rank, every rank reports the same note, closes the peer path and takes RCCL;
    two ranks sharing one GPU (no RCCL) stop instead."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cfg = {"all_ok": ("peer", (), (), False), "rank1_probe_fails": ("peer", (1,), (), False),
           "rank0_export_fails": ("peer", (), (0,), False), "rccl_asked": ("rccl", (), (), False),
           "shared_gpu_fails": ("peer", (1,), (), True)}[case]
    mp.spawn(_exchange_rank, args=(2, port, str(tmp_path), *cfg), nprocs=2, join=True)
    r = [json.load(open(tmp_path / f"x{k}.json")) for k in range(2)]
    if case == "shared_gpu_fails":
        assert all("peer exchange failed on one GPU" in x["exit"] for x in r)
        return
    assert r[0].get("note") == r[1].get("note")
    assert r[0]["kind"] == r[1]["kind"] == ("peer" if case == "all_ok" else "rccl")
    assert r[0]["n"] == r[1]["n"] == 2
    if case == "all_ok":
        assert r[0]["note"] is None and all("comm_init" not in x["calls"] for x in r)
    elif case == "rccl_asked":
        assert r[0]["note"] is None and all(x["calls"] == ["comm_init"] for x in r)
    else:
        assert "fake" in r[0]["note"]
        assert all(x["calls"][-2:] == ["peer_close", "comm_init"] for x in r)
