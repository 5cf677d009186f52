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
