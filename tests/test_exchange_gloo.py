"""The N>1 exchange path on CPU: two processes (gloo, world size 2), one partition each (the CPU
oracle stands in for the device partition), outboxes bucketed by target partition and exchanged
with DeviceExchange (the count all_gather and the all_to_all_single of the 48-byte commands: the
same calls RCCL runs on the GPUs).  The result must equal the single-process cluster driven by
exchange.route().  The GPU twin (libzbhip partitions in every rank) is
tests/test_gpu_multiprocess.py."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from helpers import MessageCluster, OracleAdapter, create_commands, string_docs
from oracle.oracle import Oracle, subscription_partition
from zeebe_amd import abi, bpmn

XML = bpmn.message_catch_process()
N = 30
P = 2


def _keys():
    return ["k-%d-%d" % (p, i) for p in range(1, P + 1) for i in range(N)]


def _bucket(ob):
    ob = np.asarray(ob, dtype=abi.XPART_DTYPE)
    counts = [int(np.sum(ob["target_partition"] == t)) for t in range(1, P + 1)]
    order = np.argsort(ob["target_partition"], kind="stable")
    return ob[order], counts


class _OraclePartition:
    """The partition surface DeviceExchange.exchange_partition drives (outbox_device_async,
    outbox_copy, submit_xparts_device, run) over the CPU oracle; "device" buffers are host memory
    (CPU tensors of the gloo path)."""

    def __init__(self, o, on_window):
        self.o = o
        self.on_window = on_window
        self.ob = abi.make_xparts(0)
        self.pending = None

    def outbox_device_async(self, counts_ptr):
        import ctypes
        self.bucketed, counts = _bucket(self.ob)
        self.ob = abi.make_xparts(0)  # handed out once
        c = np.asarray(counts, dtype=np.int32)
        ctypes.memmove(counts_ptr, c.ctypes.data, c.nbytes)
        return 0

    def outbox_copy(self, dst, first, count):
        import ctypes
        src = np.ascontiguousarray(self.bucketed[first:first + count])
        ctypes.memmove(dst, src.ctypes.data, src.nbytes)

    def submit_xparts_device(self, ptr, n):
        import ctypes
        buf = (ctypes.c_uint8 * (n * abi.XPART_DTYPE.itemsize)).from_address(ptr)
        self.pending = np.frombuffer(bytes(buf), dtype=abi.XPART_DTYPE)

    def run(self, flags=0):
        from zeebe_amd.exchange import window_from_xparts
        cmds, xp = window_from_xparts(self.pending)
        self.ob = self.on_window(cmds, xp)


def _rank_main(rank, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from zeebe_amd.exchange import DeviceExchange, window_from_xparts
    dist.init_process_group("gloo", rank=rank, world_size=P)
    ex = DeviceExchange()
    o = Oracle(partition_id=rank + 1, partition_count=P)
    o.deploy(XML)
    ids = [o.intern_string(k) for k in _keys()]
    var, name = o.intern("key"), o.intern("msg")
    log = []

    def window(phase, cmds, docs=None, xp=None):
        recs, ob = OracleAdapter.window(o, cmds, docs, xp)
        log.append([phase, [abi.record_tuple(r) for r in recs]])
        return ob

    staging = torch.empty(64 * N * abi.XPART_DTYPE.itemsize, dtype=torch.uint8)

    def exchange(phase, ob):
        part = _OraclePartition(o, lambda cmds, xp: window(phase, cmds, None, xp))
        part.ob = ob
        for _ in range(6):
            got, total = ex.exchange_partition(part, staging)
            if total == 0:
                return

    c = create_commands(N)
    c["doc_count"] = 1
    c["doc_begin"] = np.arange(N)
    ob = window("create", c, string_docs(var, ids[rank * N:(rank + 1) * N]))
    exchange("subscribe", ob)
    mine = [i for i, k in zip(ids, _keys()) if subscription_partition(k, P) == rank + 1]
    pub = abi.make_commands(len(mine))
    pub["instance"] = mine
    pub["kind"] = abi.CMD_PUBLISH
    pub["ref"] = name
    ob = window("publish", pub) if len(mine) else abi.make_xparts(0)
    exchange("correlate", ob)
    with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as f:
        json.dump({"log": log, "state": o.state(), "counters": o.counters()}, f)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_exchange_matches_single_process_cluster(tmp_path):
    mp.start_processes(_rank_main, args=(_free_port(), str(tmp_path)), nprocs=P, join=True, start_method="spawn")
    ranks = [json.load(open(tmp_path / ("rank%d.json" % r))) for r in range(P)]
    cl = MessageCluster([Oracle(partition_id=p, partition_count=P) for p in range(1, P + 1)], OracleAdapter, XML)
    keys = _keys()
    ids = cl.intern_keys(keys)
    cl.create(N, [ids[(p - 1) * N:p * N] for p in range(1, P + 1)])
    cl.publish(ids, [subscription_partition(k, P) for k in keys])
    for p in range(1, P + 1):
        want = [[ph, [list(abi.record_tuple(r)) for r in recs]] for ph, q, recs, _ in cl.log if q == p]
        assert ranks[p - 1]["log"] == want
        assert ranks[p - 1]["state"] == cl.parts[p - 1].state()
    assert sum(r["counters"]["completed_instances"] for r in ranks) == N * P
