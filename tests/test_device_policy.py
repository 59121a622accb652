"""Device selection (SURVEY 8 e): which GPU a kuma loop
thread's decoders, batches and rings use (include/kmws_gpu.h
KMWS_DEVICE_AUTO / KMWS_DEVICE_POLICY_*, kuma_amd/csrc/kmws_devmap.cpp).

The policy is a pure function of (policy, the thread's NUMA node, the GPUs'
nodes, how many threads were placed before): kmws_device_policy_pick, driven
here with synthetic node topologies, no GPU needed.  The GPU-side check (the
one-GPU box: every policy gives device 0, pins are honoured) is in
tests/test_gpu_e2e_shard.py."""
import collections

import pytest

from kuma_amd import kmws

NUMA, RR, FIRST = kmws.DEVICE_POLICY_NUMA, kmws.DEVICE_POLICY_ROUND_ROBIN, kmws.DEVICE_POLICY_FIRST
# an 8-GPU node with two sockets: GPUs 0-3 behind socket 0, 4-7 behind socket 1
TWO_SOCKETS = [0, 0, 0, 0, 1, 1, 1, 1]


def pick(policy, node, gpus, seq):
    return kmws.device_policy_pick(policy, node, gpus, seq)


def test_first_is_device_zero():
    assert [pick(FIRST, n, TWO_SOCKETS, s) for n in (-1, 0, 1) for s in range(5)] == [0] * 15


def test_round_robin_covers_every_gpu_in_thread_order():
    assert [pick(RR, 1, TWO_SOCKETS, s) for s in range(10)] == [0, 1, 2, 3, 4, 5, 6, 7, 0, 1]


def test_numa_keeps_threads_on_their_sockets_gpus():
    assert [pick(NUMA, 0, TWO_SOCKETS, s) for s in range(6)] == [0, 1, 2, 3, 0, 1]
    assert [pick(NUMA, 1, TWO_SOCKETS, s) for s in range(6)] == [4, 5, 6, 7, 4, 5]


def test_numa_falls_back_to_every_gpu():
    # the thread's node is unknown, has no GPU, or the GPUs' nodes are unknown (-1 in sysfs)
    assert [pick(NUMA, -1, TWO_SOCKETS, s) for s in range(9)] == [0, 1, 2, 3, 4, 5, 6, 7, 0]
    assert [pick(NUMA, 3, TWO_SOCKETS, s) for s in range(3)] == [0, 1, 2]
    assert [pick(NUMA, 0, [-1] * 8, s) for s in range(3)] == [0, 1, 2]


def test_kumas_loop_pools_spread_over_the_node():
    """kuma's test client runs 10 loop threads (test/client/main.cpp:20), its
    server 5 (test/server/main.cpp:22): on the two-socket node with threads
    alternating sockets, no GPU takes more than 2 of the 10, every GPU at least
    one, and a thread stays on its socket's GPUs."""
    seq = collections.Counter()
    got = []
    for t in range(10):
        node = t % 2
        got.append(pick(NUMA, node, TWO_SOCKETS, seq[node]))
        seq[node] += 1
        assert TWO_SOCKETS[got[-1]] == node
    per_gpu = collections.Counter(got)
    assert set(per_gpu) == set(range(8)) and max(per_gpu.values()) == 2
    # the server's 5 threads on socket 1 only
    assert [pick(NUMA, 1, TWO_SOCKETS, s) for s in range(5)] == [4, 5, 6, 7, 4]


def test_bad_arguments():
    assert pick(7, 0, TWO_SOCKETS, 0) == kmws.ERR_INVALID_PARAM
    assert pick(NUMA, 0, [], 0) == kmws.ERR_NOT_SUPPORTED
    assert kmws.lib().kmws_set_device_policy(9) == kmws.ERR_INVALID_PARAM
    assert kmws.lib().kmws_set_device_policy(NUMA) == kmws.OK
    assert kmws.lib().kmws_set_thread_device(-5) == kmws.ERR_INVALID_PARAM
    assert kmws.lib().kmws_set_thread_device(kmws.DEVICE_AUTO) == kmws.OK  # unpin


def test_no_device_here_fails_loudly():
    """Without a gfx950 device the calling thread has no device: AUTO entries
    fail (no CPU fallback), a pin to device 0 is refused."""
    if kmws.device_count() > 0:
        pytest.skip("a device is present")
    L = kmws.lib()
    assert L.kmws_thread_device() == kmws.ERR_NOT_SUPPORTED
    assert L.kmws_set_thread_device(0) == kmws.ERR_NOT_SUPPORTED
    assert L.kmws_thread_attach(kmws.DEVICE_AUTO) == kmws.ERR_NOT_SUPPORTED
    assert not L.kmws_rx_batch_create(kmws.DEVICE_AUTO)
    assert not L.kmws_tx_batch_create(kmws.DEVICE_AUTO)
    assert not L.kmws_host_alloc(4096, kmws.DEVICE_AUTO)
    assert not L.kmws_pipeline_create(kmws.DEVICE_AUTO, 1 << 20, 16, 3)
    with pytest.raises(kmws.KmwsError):
        kmws.handle_data_mask(b"abcd", [bytearray(b"xyz")], device=kmws.DEVICE_AUTO)
