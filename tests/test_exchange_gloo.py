"""The N>1 exchange path on CPU: two processes (gloo, world size 2), one partition each (the CPU
oracle stands in for the device partition), outboxes bucketed by target partition and exchanged
with DeviceExchange.send (all_to_all_single of counts, then of the 48-byte commands: the same calls
RCCL runs on the GPUs).  The result must equal the single-process cluster driven by
exchange.route()."""
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

    def exchange(phase, ob):
        for _ in range(6):
            bucketed, counts = _bucket(ob)
            payload = torch.from_numpy(bucketed.view(np.uint8).copy())
            inbox, got = ex.send(payload, counts)
            total = torch.tensor([got])
            dist.all_reduce(total)
            if int(total) == 0:
                return
            ob = abi.make_xparts(0)
            if got:
                xp = np.frombuffer(inbox.numpy().tobytes(), dtype=abi.XPART_DTYPE)
                cmds, xp = window_from_xparts(xp)
                ob = window(phase, cmds, None, xp)

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
