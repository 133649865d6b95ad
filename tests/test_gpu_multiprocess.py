"""Config 5 across processes on the gfx950 path: P ranks (one partition each, libzbhip handles on
cuda:0), the subscription exchange through DeviceExchange.exchange_partition -- the device outbox
buckets (zbhip_outbox_device_async), one count collective, one all-to-all of the 48-byte commands,
the received window built on the device (zbhip_submit_xparts_device).  The ranks share one GPU, so
the process group is gloo (host-staged collectives); with one GPU per rank the same code runs over
RCCL (bench.py --config msg --gpus N), exercised here at one rank over ``nccl``.

Bar: every window's records (all parity fields, keys relabelled) and the final state of every
partition equal the single-process oracle cluster driven by exchange.route()
(MessageCorrelationMultiplePartitionsTest.java:57-175 is the reference's multi-partition test;
InterPartitionCommandSenderImpl.java:51-100 the routing the exchange replaces)."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from helpers import MessageCluster, OracleAdapter, create_commands, string_docs
from oracle.oracle import Oracle, subscription_partition
from zeebe_amd import abi, bpmn

pytestmark = pytest.mark.gpu

XML = bpmn.message_catch_process()
N = 40


def _keys(P):
    return ["k-%d-%d" % (p, i) for p in range(1, P + 1) for i in range(N)]


def _rank_main(rank, P, port, out_dir, backend="gloo"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from zeebe_amd.engine import Partition
    from zeebe_amd.exchange import XPART_BYTES, DeviceExchange
    dev = torch.device("cuda", 0)
    if backend == "nccl":  # RCCL: DeviceExchange's device branch (device counts, device all-to-all)
        torch.cuda.set_device(dev)
    dist.init_process_group(backend, rank=rank, world_size=P)
    stream = torch.cuda.Stream(device=dev).cuda_stream  # one stream shared by the partitions (exchange order)
    part = Partition(partition_id=rank + 1, partition_count=P, max_instances=N, max_commands=4 * N * P,
                     max_correlation_keys=N * P, max_records_per_batch=256, stream=stream)
    part.deploy(XML)
    keys = _keys(P)
    ids = [int(x) for x in part.intern_strings(keys)]
    var, name = part.intern("key"), part.intern("msg")
    ex = DeviceExchange(max_entries=4 * N * P, device=dev)
    staging = torch.empty(6 * 4 * N * P * XPART_BYTES, dtype=torch.uint8, device=dev)
    log = []

    def drained(phase):
        recs = part.drain()
        assert part.fallback() == []
        log.append([phase, [abi.record_tuple(r) for r in recs]])

    def exchange(phase):
        for _ in range(8):
            got, total = ex.exchange_partition(part, staging, 0)
            if total == 0:
                return
            if got:
                drained(phase)
        raise AssertionError("exchange did not quiesce")

    c = create_commands(N)
    c["doc_count"] = 1
    c["doc_begin"] = np.arange(N)
    part.submit(c, string_docs(var, ids[rank * N:(rank + 1) * N]))
    part.run()
    drained("create")
    exchange("subscribe")
    mine = [i for i, k in zip(ids, keys) if subscription_partition(k, P) == rank + 1]
    if mine:
        pub = abi.make_commands(len(mine))
        pub["instance"] = mine
        pub["kind"] = abi.CMD_PUBLISH
        pub["ref"] = name
        part.submit(pub)
        part.run()
        drained("publish")
    else:  # nothing published here: the outbox of the last run is already handed out
        pass
    exchange("correlate")
    torch.cuda.synchronize()
    with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as f:
        json.dump({"log": log, "state": part.state()}, f)
    part.close()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("P,backend", [(2, "gloo"), (8, "gloo"), (1, "nccl")])
def test_gpu_ranks_exchange_matches_oracle_cluster(P, backend, tmp_path):
    """(P = 1 over ``nccl``: the RCCL branch of DeviceExchange -- counts gathered and commands
    exchanged as device tensors -- on the one GPU of the test box; the gloo cases share it.)"""
    mp.start_processes(_rank_main, args=(P, _free_port(), str(tmp_path), backend), nprocs=P, join=True,
                       start_method="spawn")
    ranks = [json.load(open(tmp_path / ("rank%d.json" % r))) for r in range(P)]
    cl = MessageCluster([Oracle(partition_id=p, partition_count=P) for p in range(1, P + 1)], OracleAdapter, XML)
    keys = _keys(P)
    ids = cl.intern_keys(keys)
    cl.create(N, [ids[(p - 1) * N:p * N] for p in range(1, P + 1)])
    cl.publish(ids, [subscription_partition(k, P) for k in keys])
    for p in range(1, P + 1):
        want = [[ph, [list(abi.record_tuple(r)) for r in recs]] for ph, q, recs, _ in cl.log if q == p]
        got = ranks[p - 1]["log"]
        assert [g[0] for g in got] == [w[0] for w in want], p
        for (ph, g), (_, w) in zip(got, want):
            assert g == w, (p, ph)
        assert ranks[p - 1]["state"] == cl.parts[p - 1].state(), p
    # PROCESS ELEMENT_COMPLETED records drained on the ranks: every instance of the cluster completed
    done = sum(1 for r in ranks for _, recs in r["log"] for t in recs
               if t[3] == abi.VT_PROCESS_INSTANCE and t[4] == 5 and t[10] == 0 and t[2] == abi.RT_EVENT)
    assert done == N * P
