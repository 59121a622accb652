"""GPU: the sharded HIP path of bench.py (BASELINE configs[4], SURVEY 8 e).

`bench.py --gpus 2 --dist-backend gloo` starts its two rank processes itself
(one GPU per rank; on a one-GPU box both share it), each rank generates its
own shard of a fixed job on the device, unmasks it with the product kernels
in resident sub-batches, and verifies every byte with the device checker.
The test reads rank 0's JSON line: two ranks, contiguous shards covering the
job, sub-batches covering each shard, no mismatches, a clean status word."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout[-2000:]  # ONE JSON line, whatever the ranks' libraries print
    return json.loads(lines[0])


@pytest.mark.parametrize("job,max_batch", [(65536, 16384), (50001, 20000)])
def test_bench_two_ranks_shard_the_job(job, max_batch):
    d = run_bench("--gpus", "2", "--dist-backend", "gloo", "--job-frames", str(job), "--max-batch-frames",
                  str(max_batch), "--steps", "3", "--warmup", "1", "--cpu-seconds", "0", "--e2e-gib", "0")
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["verify"]["byte_mismatches"] == 0 and d["verify"]["status_word"] == 0
    ranks = sorted(d["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == [0, 1]
    assert ranks[0]["frames"][0] == 0 and ranks[-1]["frames"][1] == job
    assert ranks[0]["frames"][1] == ranks[1]["frames"][0]
    for r in ranks:
        subs = r["sub_batches"]
        assert subs[0][0] == r["frames"][0] and subs[-1][1] == r["frames"][1]
        assert all(a[1] == b[0] for a, b in zip(subs, subs[1:]))
        assert all(hi - lo <= max_batch for lo, hi in subs)
        assert r["byte_mismatches"] == 0
    assert len({len(r["sub_batches"]) for r in ranks}) == 1  # the barriers pair up
    assert d["value"] > 0 and d["config"]["total_frames"] == job


def test_bench_one_gpu_small_batch_plain_rate():
    """N = 1 weak scaling on a small batch, default placement: the timed batch
    is a plain allocation, so the plain rate is the headline's own."""
    d = run_bench("--frames", "16384", "--steps", "3", "--warmup", "1", "--cpu-seconds", "0", "--cfg5-anchor", "0",
                  "--e2e-gib", "0")
    assert d["n_gpus"] == 1 and d["scaling"] == "weak" and d["verify"]["byte_mismatches"] == 0
    assert d["config"]["placement"]["kind"] == "plain torch.empty"
    assert d["roofline"]["frac_plain"] == d["roofline"]["frac"] > 0  # the timed batch is the plain allocation


CFG5_FRAMES = 10485760  # BASELINE configs[4]: 10 M x 64 KiB = 640 GiB
CFG5_BATCH = 1310720    # bench.py --max-batch-frames default: 80 GiB resident per sub-batch
_cfg5 = {}


def _check_cfg5(d, world):
    assert d["n_gpus"] == world and d["scaling"] == "strong"
    assert d["config"]["total_frames"] == CFG5_FRAMES and d["config"]["frame_len"] == 65536
    _check_cfg5_ranks(d, world)


def _check_cfg5_ranks(d, world):
    assert d["verify"]["byte_mismatches"] == 0 and d["verify"]["status_word"] == 0
    ranks = sorted(d["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == list(range(world))
    assert ranks[0]["frames"][0] == 0 and ranks[-1]["frames"][1] == CFG5_FRAMES
    assert all(a["frames"][1] == b["frames"][0] for a, b in zip(ranks, ranks[1:]))  # contiguous shards
    for r in ranks:
        subs = r["sub_batches"]
        assert len(subs) == 8 // world
        assert subs[0][0] == r["frames"][0] and subs[-1][1] == r["frames"][1]
        assert all(a[1] == b[0] for a, b in zip(subs, subs[1:]))
        assert all(hi - lo == CFG5_BATCH for lo, hi in subs)
        assert r["byte_mismatches"] == 0
    assert d["value"] > 0


@pytest.mark.timeout(600)
def test_cfg5_job_anchor_at_one_gpu():
    """the N = 1 line (cfg2, here on a small batch) also carries
    `cfg5_job`, BASELINE configs[4]'s real job -- 10,485,760 x 64 KiB frames as 8
    resident sub-batches of 1,310,720 frames (80 GiB), each generated on the
    device, timed as the N > 1 lines time their ranks' sub-batches, verified
    byte for byte: the same-job anchor of the 1 -> 8 curve."""
    d = run_bench("--gpus", "1", "--frames", "16384", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0",
                  "--e2e-gib", "0", timeout=600)
    assert d["n_gpus"] == 1 and d["scaling"] == "weak" and d["config"]["total_frames"] == 16384
    c = d["cfg5_job"]
    assert c["total_frames"] == CFG5_FRAMES and c["sub_batches"] == 8 and c["resident_batch_frames"] == CFG5_BATCH
    assert c["scaling"] == "strong" and c["frame_len"] == 65536
    _check_cfg5_ranks(c, 1)
    assert d["verify"]["byte_mismatches"] == 0
    _cfg5[1] = c["value"]


@pytest.mark.timeout(600)
def test_cfg5_full_job_two_ranks_share_the_gpu():
    """The same job at --gpus 2 (gloo harness, both ranks on the one GPU of the
    box): 4 sub-batches per rank over contiguous shards, every byte verified;
    the two ranks share one GPU's HBM, so the aggregate must stay within 10 %
    of the N = 1 line's cfg5_job value, the same job timed the same way
    (nothing is lost to the partition or the harness)."""
    d = run_bench("--gpus", "2", "--dist-backend", "gloo", "--job-frames", str(CFG5_FRAMES), "--steps", "2",
                  "--warmup", "1", "--cpu-seconds", "0", "--e2e-gib", "0", timeout=600)
    _check_cfg5(d, 2)
    assert d["cfg5_job"] is None  # the N > 1 headline is the job itself
    if 1 in _cfg5:
        assert abs(d["value"] / _cfg5[1] - 1) <= 0.10, (d["value"], _cfg5[1])
