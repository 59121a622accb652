"""CPU checks of bench.py's harness pieces (no GPU): the cfg1 wire image the
benchmark feeds is a valid masked stream that kuma's decoder (oracle)
decodes back to the plain payloads, and the placement/sub-batch arithmetic
the headline run relies on."""
import json
import os
import subprocess
import sys

import numpy as np

from kuma_amd import shard
from oracle import oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cfg1_cpu_baseline_runs_without_gpu():
    """bench.py --config cfg1 on a host without a GPU: the cpu_baseline leg
    (kuma's decoder restated in oracle/) decodes the whole stream; no product
    numbers are reported (no CPU fallback)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "cfg1", "--steps", "2"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["config"] == "cfg1" and d["frames"] == 1000 and d["wire_bytes"] == 1000 * (8 + 4096)
    assert d["cpu_baseline"]["GiB_s"] > 0 and d["cpu_baseline"]["cores"] == 1
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if not has_gpu:
        assert not any(k.startswith("product") for k in d)


def test_cfg1_wire_decodes_to_plain_payloads():
    """The wire construction used by bench.run_cfg1 (81 fe 10 00 key | payload ^ key)
    equals the oracle's encodeFrameHeader + mask for every frame."""
    n, L = 8, 4096
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    payload = (0x20 + rng.integers(0, 95, size=n * L)).astype(np.uint8)
    kb = keys.view(np.uint8).reshape(n, 4)
    frames = np.empty((n, 8 + L), dtype=np.uint8)
    frames[:, :4] = np.array([0x81, 0xFE, L >> 8, L & 0xFF], dtype=np.uint8)
    frames[:, 4:8] = kb
    frames[:, 8:] = payload.reshape(n, L) ^ np.tile(kb, L // 4)
    want = b"".join(orc.encode_header(orc.Hdr(fin=1, opcode=1, mask=1, maskey=bytes(kb[i]), length=L)) +
                    orc.mask_bytes(bytes(kb[i]), payload[i * L:(i + 1) * L].tobytes()) for i in range(n))
    assert frames.tobytes() == want
    rets, fr = orc.decode_chunks(want, orc.SERVER, 65536)
    assert rets[-1] == 0 and [f.payload for f in fr] == [payload[i * L:(i + 1) * L].tobytes() for i in range(n)]


def test_placement_slack_and_offsets():
    """place_batch's slack rule: multiples of 16 GiB, at most 1.5 x the batch and
    what fits beside it; offsets 0, 16, ... GiB inside the arena."""
    sys.path.insert(0, ROOT)
    import bench
    step = bench.PLACEMENT_STEP
    assert step == 16 << 30

    def slack(span, free, want=96 << 30):
        return bench.placement_slack(span, free, want)

    assert slack(64 << 30, 280 << 30) == 96 << 30            # cfg2 on a 288 GB GPU: 160 GiB arena
    assert slack(80 << 30, 280 << 30) == 96 << 30            # cfg5 resident batch: 176 GiB arena
    assert slack(16 << 30, 280 << 30) == 16 << 30            # small batches: little slack
    assert slack(4 << 30, 280 << 30) < step                  # too small to probe: plain allocation
    assert slack(64 << 30, 100 << 30) == 16 << 30            # memory already in use: what fits
    assert slack(64 << 30, 60 << 30) == 0                    # not even the batch fits beside: no probe
    offsets = list(range(0, (96 << 30) + 1, step))
    assert len(offsets) == 7 and offsets[-1] + (64 << 30) == 160 << 30


def test_cfg5_sub_batches_per_gpu_count():
    for world, nb in ((1, 8), (2, 4), (4, 2), (8, 1)):
        n, bs = shard.sub_batches(10485760, 0, world, 1310720)
        assert len(bs) == nb and n == 1310720


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def test_gpus_world_size_mismatch_is_refused():
    """Under a launcher, --gpus N must equal WORLD_SIZE (one rank per GPU)."""
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


def test_gpus_n_starts_n_ranks_itself():
    """bench.py --gpus 2 without WORLD_SIZE starts 2 rank processes (torchrun's
    environment, 127.0.0.1 rendezvous).  Without a GPU every rank refuses to run
    (no CPU fallback) and the launcher returns a non-zero status; the GPU form
    of this check is tests/test_gpu_bench_sharded.py."""
    if _has_gpu():
        return
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode != 0
    assert r.stderr.count("no GPU visible") == 2, r.stderr


def test_launch_ranks_environment(tmp_path):
    """launch_ranks gives rank r RANK=LOCAL_RANK=r, WORLD_SIZE=N and one shared
    127.0.0.1 rendezvous port, re-running the same script with the same argv."""
    script = tmp_path / "probe.py"
    script.write_text(
        "import os, sys, json\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import bench\n"
        "if 'WORLD_SIZE' not in os.environ:\n"
        "    bench.__file__ = __file__\n"
        "    sys.exit(bench.launch_ranks(3))\n"
        "print(json.dumps({k: os.environ[k] for k in ('RANK','LOCAL_RANK','WORLD_SIZE','MASTER_ADDR','MASTER_PORT')}"
        " | {'argv': sys.argv[1:]}))\n")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(script), "--x", "1"], capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode == 0, r.stderr
    # only rank 0's JSON line reaches stdout (the contract's one line); the other
    # ranks' output is forwarded to stderr
    out = r.stdout.strip().splitlines()
    assert len(out) == 1 and json.loads(out[0])["RANK"] == "0", r.stdout
    rows = [json.loads(x) for x in out + [y for y in r.stderr.splitlines() if y.startswith("{")]]
    assert sorted(int(x["RANK"]) for x in rows) == [0, 1, 2]
    assert all(x["RANK"] == x["LOCAL_RANK"] and x["WORLD_SIZE"] == "3" and x["MASTER_ADDR"] == "127.0.0.1"
               for x in rows)
    assert len({x["MASTER_PORT"] for x in rows}) == 1 and all(x["argv"] == ["--x", "1"] for x in rows)


def test_cpu_baseline_cores_are_the_effective_count(monkeypatch):
    """the CPU baseline runs min(affinity, ceil(cgroup quota))
    threads and reports that number as `cores`, the 1-thread rate beside it,
    and says the port is uncalibrated against a reference build."""
    sys.path.insert(0, ROOT)
    import bench
    for (aff, quota), want in (((256, 16.0), 16), ((256, 15.5), 16), ((8, 16.0), 8), ((64, None), 64),
                               ((4, 0.5), 1)):
        monkeypatch.setattr(bench, "host_cores", lambda a=aff, q=quota: (a, q))
        assert bench.effective_cores() == want
    monkeypatch.setattr(bench, "host_cores", lambda: (256, 2.0))
    cb = bench.cpu_baseline(0.2, bench.effective_cores(), 4096, 1)
    assert cb["cores"] == 2 and cb["affinity_cores"] == 256 and cb["cgroup_cpu_quota_cores"] == 2.0
    assert cb["value"] > 0 and cb["single_core_GiB_s"] > 0 and "not calibrated" in cb["sample"]


def test_traffic_from_profile_takes_the_newest_record(tmp_path):
    """`traffic` is the newest PMC record for the bench's
    schedule by the time stamped in it, not the last file name in sort order;
    records without a stamp rank below stamped ones; another schedule's
    record is used only when none matches."""
    import json
    import bench
    def rec(name, when, val, sched=536870914):
        t = {"kernel": bench.UNMASK_KERNEL, "frames": 8, "frame_len": 64, "schedule": sched,
             "hbm_bytes_per_launch": val}
        if when:
            t["measured_at"] = when
        (tmp_path / name).write_text(json.dumps(t))
    rec("r09_pmc_traffic.json", "2026-10-17T03:00:00+00:00", 1.0)
    rec("r05b_pmc_traffic.json", "2026-10-18T09:00:00+00:00", 2.0)
    rec("r07_pmc_traffic.json", None, 3.0)
    rec("r08_pmc_traffic.json", "2026-10-19T09:00:00+00:00", 4.0, sched=5)
    f = bench.traffic_from_profile
    assert f(8, 64, bench.UNMASK_KERNEL, 536870914, profiles_dir=str(tmp_path)) == 2.0
    assert f(8, 64, bench.UNMASK_KERNEL, 7, profiles_dir=str(tmp_path)) == 4.0  # no match: newest of any
    assert f(8, 65, bench.UNMASK_KERNEL, 7, profiles_dir=str(tmp_path)) is None
