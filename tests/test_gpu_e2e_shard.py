"""GPU: the host-resident path on N ranks (SURVEY 8 e) and the
device selection policy on a real device.

`bench.py --config e2e --gpus 2 --dist-backend gloo` starts two rank processes
(on the one-GPU box both share the GPU and its PCIe link): each rank writes
its own shard of masked 64 KiB frames into pinned host memory
(kmws_host_alloc), unmasks it in place end to end through its own
kmws_pipeline (pinned H2D -> unmask kernel -> D2H), and verifies every byte on
the device.  No data-path collective."""
import ctypes
import json
import os
import subprocess
import sys
import threading

import pytest

from kuma_amd import kmws
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [1, 2])
def test_e2e_each_rank_its_own_pipeline(world):
    d = run_bench("--config", "e2e", "--gpus", str(world), "--dist-backend", "gloo", "--e2e-gib", "0.5",
                  "--steps", "3", "--warmup", "1")
    assert d["n_gpus"] == world and d["scaling"] == "weak" and d["metric"].startswith("GiB/s host-resident")
    assert d["verify"]["ok"] and d["verify"]["byte_mismatches"] == 0
    ranks = sorted(d["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == list(range(world))
    n = d["config"]["frames_per_gpu"]
    assert n == int(0.5 * 2**30) // (65536 + 14)
    for r in ranks:
        assert r["byte_mismatches"] == 0 and r["payload_GiB_s"] > 0
        assert r["raw_h2d_GiB_s"] > 0 and r["raw_d2h_GiB_s"] > 0
    assert d["value"] > 0 and d["pcie"]["bytes_per_step_per_gpu"] == 2 * n * (65536 + 14)


def test_default_bench_line_carries_e2e_host():
    """The driver's N-GPU bench line records the host-resident rate beside the
    headline (e2e_host), so the 1 -> 8 scaling runs measure it too."""
    d = run_bench("--frames", "16384", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0", "--cfg5-anchor", "0",
                  "--e2e-gib", "0.25")
    e = d["e2e_host"]
    assert "error" not in e, e
    assert e["verify"]["ok"] and e["n_gpus"] == 1 and e["value"] > 0


def test_device_policy_on_the_box():
    """Every policy gives a new thread a valid device (one GPU here: 0); a pin is
    honoured and a pin past the last device refused; AUTO objects work."""
    ndev = kmws.device_count()
    got = {}

    def probe(policy):
        kmws.set_device_policy(policy)
        got[policy] = kmws.thread_device()

    for p in (kmws.DEVICE_POLICY_NUMA, kmws.DEVICE_POLICY_ROUND_ROBIN, kmws.DEVICE_POLICY_FIRST):
        t = threading.Thread(target=probe, args=(p,))
        t.start()
        t.join()
    kmws.set_device_policy(kmws.DEVICE_POLICY_NUMA)
    assert all(0 <= d < ndev for d in got.values()) and got[kmws.DEVICE_POLICY_FIRST] == 0
    L = kmws.lib()
    res = {}

    def pinned():
        res["pin0"] = L.kmws_set_thread_device(0)
        res["dev"] = L.kmws_thread_device()
        res["pin_bad"] = L.kmws_set_thread_device(ndev)
        res["attach"] = L.kmws_thread_attach(kmws.DEVICE_AUTO)
        node = ctypes.c_int(-2)
        res["node"] = (L.kmws_device_numa_node(0, ctypes.byref(node)), node.value)

    t = threading.Thread(target=pinned)
    t.start()
    t.join()
    assert res["pin0"] == 0 and res["dev"] == 0 and res["pin_bad"] == kmws.ERR_NOT_SUPPORTED
    assert res["attach"] >= 0 or res["attach"] == kmws.ERR_NOT_SUPPORTED  # a slot, or all 16 taken
    assert res["node"][0] == 0 and res["node"][1] >= -1
    # a decoder and a host mask on the thread's device (AUTO), exact against the oracle
    key = b"\x37\xfa\x21\x3d"
    data = bytes(range(256)) * 33
    h = kmws.WSHandler(kmws.SERVER, device=kmws.DEVICE_AUTO)
    frames = []
    h.setFrameCallback(lambda hd, p: frames.append(p))
    wire = orc.encode_header(orc.Hdr(fin=1, opcode=2, mask=1, maskey=key, length=len(data))) + \
        orc.mask_bytes(key, data)
    assert h.handleData(bytearray(wire)) == 0 and frames == [data]
    buf = bytearray(data)
    kmws.handle_data_mask(key, [buf], device=kmws.DEVICE_AUTO)
    assert bytes(buf) == orc.mask_bytes(key, data)


def test_two_rank_bench_line_carries_e2e_host():
    """The N > 1 line (here two gloo ranks on the one GPU, a small strong-scaling
    job) carries the host-resident leg too: both ranks' shards verified."""
    d = run_bench("--gpus", "2", "--dist-backend", "gloo", "--job-frames", "65536", "--max-batch-frames", "16384",
                  "--steps", "2", "--warmup", "1", "--cpu-seconds", "0", "--e2e-gib", "0.25")
    e = d["e2e_host"]
    assert "error" not in e, e
    assert e["n_gpus"] == 2 and len(e["ranks"]) == 2 and e["verify"]["ok"]
    assert d["verify"]["byte_mismatches"] == 0 and d["cfg5_job"] is None
