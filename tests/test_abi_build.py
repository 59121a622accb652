"""The C ABI header compiles as C99 and C++17 and a C++ program links and
runs against libkmws_gpu.so (the way kuma's C++ would consume it)."""
import os
import subprocess

import pytest

from kuma_amd import build as kb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")


def test_header_is_plain_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "kmws_gpu.h"\nint main(void){ kmws_desc d; (void)d; '
                   'return kmws_make_flags(1,0,0,0,2,1) == 0x182 ? 0 : 1; }\n')
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Werror", "-pedantic", "-I", INC, "-fsyntax-only",
                           str(src)])


def _build_and_run(tmp_path):
    lib = kb.build()
    exe = tmp_path / "abi_smoke"
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-I", INC,
                           os.path.join(ROOT, "tests", "cpp", "abi_smoke.cpp"),
                           "-L", os.path.dirname(lib), "-lkmws_gpu",
                           "-Wl,-rpath," + os.path.dirname(lib), "-o", str(exe)])
    return subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)


def test_cpp_consumer_host_paths(tmp_path):
    r = _build_and_run(tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout


@pytest.mark.gpu
def test_cpp_consumer_on_gpu(tmp_path):
    r = _build_and_run(tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr


def _build_adapter(tmp_path, sanitize=False):
    """tests/cpp/wshandler_adapter.cpp: include/kmws_wshandler.hpp (the C++
    WSHandler drop-in) driven like WebSocket::Impl drives kuma's WSHandler."""
    lib = kb.build()
    exe = tmp_path / ("wsa_asan" if sanitize else "wsa")
    flags = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer"] if sanitize else ["-O2"]
    subprocess.check_call(["g++", "-std=c++14", "-Wall", "-Wextra", "-Werror", *flags, "-I", INC,
                           os.path.join(ROOT, "tests", "cpp", "wshandler_adapter.cpp"),
                           "-L", os.path.dirname(lib), "-lkmws_gpu",
                           "-Wl,-rpath," + os.path.dirname(lib), "-o", str(exe)])
    return exe


def _no_device() -> bool:
    from kuma_amd import kmws
    return kmws.lib().kmws_device_count() == 0


def test_wshandler_adapter_host(tmp_path):
    """Header pack, CLIENT-mode decode, byte-at-a-time returns, CLOSE, reset and a
    callback that deletes its handler (under ASan/UBSan); without a device a
    masked frame must fail loudly (no CPU fallback)."""
    exe = _build_adapter(tmp_path, sanitize=True)
    mode = "nogpu" if _no_device() else ""
    r = subprocess.run([str(exe), mode], capture_output=True, text=True, timeout=120,
                       env={**os.environ, "ASAN_OPTIONS": "detect_leaks=0"})
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_wshandler_adapter_on_gpu(tmp_path):
    """SERVER-mode masked frames unmasked in place on the GPU, the a-2 chain
    vector, and a 16-fragment client message (a-10/a-12) decoded back."""
    exe = _build_adapter(tmp_path)
    r = subprocess.run([str(exe), "gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


def _build_loopback(tmp_path):
    """tests/cpp/loopback_cfg1.cpp: BASELINE configs[0] over a loopback TCP socket,
    kmws (GPU) or kuma's codec restated in oracle/ (CPU) on both ends."""
    lib = kb.build()
    from oracle import oracle as orc
    orc.build()
    odir = os.path.join(ROOT, "oracle")
    exe = tmp_path / "loopback_cfg1"
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", "-I", INC,
                           os.path.join(ROOT, "tests", "cpp", "loopback_cfg1.cpp"),
                           "-L", os.path.dirname(lib), "-lkmws_gpu", "-L", odir, "-lkmws_oracle", "-lpthread",
                           "-Wl,-rpath," + os.path.dirname(lib), "-Wl,-rpath," + odir, "-o", str(exe)])
    return exe


def test_loopback_cfg1_cpu_codec(tmp_path):
    import json
    r = subprocess.run([str(_build_loopback(tmp_path)), "cpu", "2"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["verified"] and d["frames"] == 1000


def test_loopback_cfg1_cpu_codec_three_connections(tmp_path):
    """Three client / server loop-thread pairs at once, 1,000 frames each."""
    import json
    exe = _build_loopback(tmp_path)
    for mode in ("cpu", "replay_cpu", "sink_cpu"):  # replay: clients replay a masked image; sink: no decode
        r = subprocess.run([str(exe), mode, "2", "16", "0", "0", "3"], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["verified"] and d["connections"] == 3 and d["mode"] == mode


@pytest.mark.gpu
def test_loopback_cfg1_gpu_codec(tmp_path):
    """1,000 masked frames client -> server over loopback through kmws_tx_batch and
    the deferred receive batch on a pinned ring: every payload delivered intact."""
    import json
    r = subprocess.run([str(_build_loopback(tmp_path)), "gpu", "2"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["verified"] and d["frames"] == 1000


@pytest.mark.gpu
def test_loopback_cfg1_sync_member_swap(tmp_path):
    """The plain member swap over loopback: the server's drop-in decodes each
    read synchronously (resident worker), the client masks each send with the
    drop-in's static handleDataMask; every payload delivered intact, in order."""
    import json
    r = subprocess.run([str(_build_loopback(tmp_path)), "sync", "2"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["verified"] and d["frames"] == 1000 and d["mode"] == "sync"


@pytest.mark.gpu
def test_loopback_cfg1_adapter_batched(tmp_path):
    """The drop-in in batched mode over loopback: kmws::BasicWSHandler with an
    RxLoop (asynchronous submit / poll once per loop iteration) on the server,
    submitted tx generations on the client; every payload delivered intact, in
    order, at 64 KiB and 256 KiB per loop iteration."""
    import json
    exe = _build_loopback(tmp_path)
    for group in ("16", "64"):
        r = subprocess.run([str(exe), "adapter", "2", group], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["verified"] and d["frames"] == 1000 and d["mode"] == "adapter"


@pytest.mark.gpu
def test_loopback_cfg1_four_connections_share_the_resident_worker(tmp_path):
    """Four connections at once, each with its own client and server loop thread
    (eight threads holding resident slots): the adapter, the loop-batched mode,
    the synchronous member swap and the adapter's server alone (replay_adapter:
    clients replay a pre-built masked wire image) deliver every payload of every
    connection intact."""
    import json
    exe = _build_loopback(tmp_path)
    for mode in ("adapter", "gpu", "sync", "replay_adapter", "sink_adapter"):
        r = subprocess.run([str(exe), mode, "2", "16", "0", "0", "4"], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["verified"] and d["connections"] == 4 and d["mode"] == mode


def _build_sync(tmp_path):
    """tests/cpp/sync_cfg1.cpp: the synchronous drop-in vs
    kuma's codec restated in oracle/, in process, one call per 64 KiB read / per send."""
    lib = kb.build()
    from oracle import oracle as orc
    orc.build()
    odir = os.path.join(ROOT, "oracle")
    exe = tmp_path / "sync_cfg1"
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", "-I", INC,
                           os.path.join(ROOT, "tests", "cpp", "sync_cfg1.cpp"),
                           "-L", os.path.dirname(lib), "-lkmws_gpu", "-L", odir, "-lkmws_oracle", "-lpthread",
                           "-Wl,-rpath," + os.path.dirname(lib), "-Wl,-rpath," + odir, "-o", str(exe)])
    return exe


def test_sync_program_builds(tmp_path):
    assert _build_sync(tmp_path).exists()


@pytest.mark.gpu
def test_sync_cfg1_resident_drop_in(tmp_path):
    """cfg1 decoded synchronously per 64 KiB read and handleDataMask per send,
    through the resident worker and through a launch per call: every payload
    and masked buffer exact (speed is recorded by tools/bench_configs.py)."""
    import json
    r = subprocess.run([str(_build_sync(tmp_path)), "2"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    rows = [json.loads(x) for x in r.stdout.strip().splitlines()]
    assert all(x["verified"] for x in rows)
    assert {(x["case"], x["codec"]) for x in rows} >= {("decode_sync", "kmws_resident"), ("decode_sync", "kmws_launch"),
                                                       ("mask_sync", "kmws_resident")}


def _build_rx_flush(tmp_path):
    """tests/cpp/rx_flush_bench.cpp: one loop iteration's receive batch timed
    alone (flush on the resident worker, submit + poll, worker off)."""
    lib = kb.build()
    exe = tmp_path / "rx_flush_bench"
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", "-I", INC,
                           os.path.join(ROOT, "tests", "cpp", "rx_flush_bench.cpp"),
                           "-L", os.path.dirname(lib), "-lkmws_gpu", "-lpthread",
                           "-Wl,-rpath," + os.path.dirname(lib), "-o", str(exe)])
    return exe


def test_rx_flush_bench_builds(tmp_path):
    assert _build_rx_flush(tmp_path).exists()


@pytest.mark.gpu
def test_rx_flush_bench_every_mode_exact(tmp_path):
    """Every mode delivers every frame unmasked (the program exits non-zero on
    a wrong byte); small jobs go to the resident worker, the switched-off mode
    adds no worker job."""
    import json
    r = subprocess.run([str(_build_rx_flush(tmp_path)), "200", "4", "4096"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    rows = [json.loads(x) for x in r.stdout.strip().splitlines()]
    assert [x["mode"] for x in rows] == ["flush", "submitpoll", "noresident", "flush", "submitpoll"]
    assert all(x["bad"] == 0 and x["delivered"] == 250 * 4 for x in rows)
    assert rows[0]["resident_jobs"] >= 250 and rows[2]["resident_jobs"] == rows[1]["resident_jobs"]


def _build_txloop(tmp_path, testhooks=False):
    """tests/cpp/txloop_check.cpp: kmws::TxLoop against kuma's send path restated in oracle/
    (testhooks: linked against the test build, kuma_amd/build.py TEST_DEFINES)."""
    lib = kb.build()
    link = ["-L", os.path.dirname(lib), "-lkmws_gpu"]
    if testhooks:
        lib = kb.build_test_variants()[0]
        link = [os.path.abspath(lib)]
    from oracle import oracle as orc
    orc.build()
    odir = os.path.join(ROOT, "oracle")
    exe = tmp_path / ("txloop_check_th" if testhooks else "txloop_check")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", "-I", INC,
                           os.path.join(ROOT, "tests", "cpp", "txloop_check.cpp"),
                           *link, "-L", odir, "-lkmws_oracle",
                           "-Wl,-rpath," + os.path.dirname(lib), "-Wl,-rpath," + odir, "-o", str(exe)])
    return exe


def test_txloop_program_builds(tmp_path):
    assert _build_txloop(tmp_path).exists()


@pytest.mark.gpu
def test_txloop_matches_kuma_send_path(tmp_path):
    """kmws::TxLoop (sendWsFrame's batched replacement) over three
    connections of one loop, masked and unmasked frames, chains, empty payloads,
    payloads larger than its pinned ring, a ring that wraps: every connection's
    bytes equal kuma's frames (oracle) in send order; callers' buffers untouched."""
    import json
    exe = _build_txloop(tmp_path)
    for seed in ("1", "2", "3"):
        r = subprocess.run([str(exe), seed, "3000"], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["exact"] and d["callers_buffers_changed"] == 0 and d["larger_than_ring"] > 0


@pytest.mark.gpu
def test_txloop_mask_failure_drops_the_generation(tmp_path):
    """a TxLoop generation whose mask fails is never written.  Test
    build: an 80 ms stall is withdrawn and launched (exact); a 400 ms stall
    outlives timeout + drain, the flush returns KMWS_ERR_TIMEOUT, both of the
    generation's frames are dropped (no masked header with a plain payload goes
    out), their connections report -6 and later sends are refused."""
    import json
    r = subprocess.run([str(_build_txloop(tmp_path, testhooks=True)), "timeout"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["exact"] and d["flush"] == [1, 2, -6] and d["dropped"] == 2 and d["conn_results"] == [-6, -6]


def _build_thread_exit(tmp_path):
    """tests/cpp/thread_exit_check.cpp: loop threads exiting with frames queued
    while other threads claim resident slots."""
    lib = kb.build()
    from oracle import oracle as orc
    orc.build()
    odir = os.path.join(ROOT, "oracle")
    exe = tmp_path / "thread_exit_check"
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", "-I", INC,
                           os.path.join(ROOT, "tests", "cpp", "thread_exit_check.cpp"),
                           "-L", os.path.dirname(lib), "-lkmws_gpu", "-L", odir, "-lkmws_oracle", "-lpthread",
                           "-Wl,-rpath," + os.path.dirname(lib), "-Wl,-rpath," + odir, "-o", str(exe)])
    return exe


def test_thread_exit_program_builds(tmp_path):
    assert _build_thread_exit(tmp_path).exists()


@pytest.mark.gpu
def test_thread_exit_with_queued_frames_against_live_claimers(tmp_path):
    """VERDICT r05 #1.  20 rounds of 8 loop threads that each queue masked frames
    on a receive and a send loop and exit without flushing (half through
    RxLoop / TxLoop::forThisThread, half holding raw batches in a thread_local
    made before their first job, whose flush runs after the thread's exit hook),
    while 8 other threads keep starting short-lived threads that claim slots and
    mask 4 KiB buffers.  Every payload received, every frame written and every
    masked buffer equals the oracle's; no post lands on a slot its thread does
    not hold; the raw threads' late flushes launched (late posts > 0)."""
    import json
    r = subprocess.run([str(_build_thread_exit(tmp_path)), "20", "8", "8"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["exact"] and d["bad_threads"] == 0 and d["mask_bad"] == 0, d
    assert d["unowned_posts"] == 0 and d["late_posts"] > 0, d
    q = d["frames_queued_at_exit"]
    assert q["rx_pending"] > 0 and q["tx_pending"] > 0, d
    assert d["exited_threads"] == 160 and d["masks"] > 0, d
