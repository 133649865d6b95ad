"""Debug: the multi-process exchange with per-round diagnostics (scratch, not a test)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import torch.multiprocessing as mp
import test_gpu_multiprocess as T
from zeebe_amd import exchange as X

orig = X.DeviceExchange.exchange_partition
def traced(self, part, staging, flags=0):
    got, total = orig(self, part, staging, flags)
    print("rank", self.rank, "round", self.rounds, "got", got, "total", total, flush=True)
    return got, total
X.DeviceExchange.exchange_partition = traced

if __name__ == "__main__":
    import tempfile, json
    d = tempfile.mkdtemp()
    mp.start_processes(T._rank_main, args=(2, T._free_port(), d), nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        j = json.load(open(os.path.join(d, "rank%d.json" % r)))
        print(r, [(ph, len(x)) for ph, x in j["log"]])
    from helpers import MessageCluster, OracleAdapter
    from oracle.oracle import Oracle, subscription_partition
    P = 2
    cl = MessageCluster([Oracle(partition_id=p, partition_count=P) for p in range(1, P + 1)], OracleAdapter, T.XML)
    keys = T._keys(P)
    ids = cl.intern_keys(keys)
    cl.create(T.N, [ids[(p - 1) * T.N:p * T.N] for p in range(1, P + 1)])
    cl.publish(ids, [subscription_partition(k, P) for k in keys])
    print("oracle", [(ph, q, len(recs), len(ob)) for ph, q, recs, ob in cl.log])
