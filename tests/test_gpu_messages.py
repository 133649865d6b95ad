"""Config 5 on the gfx950 executor: message catch events correlated across partitions.

P partitions run in one process on cuda:0 (one libzbhip handle each, its own stream); the
exchange between them is the host routing of the outboxes (zeebe_amd.exchange.route), the same
order the CPU oracle cluster uses.  Bar: every window's records (all parity fields, keys
relabelled), every outbox entry and the exported state of every partition bit-exact against the
oracle cluster; App. A.5 sequences for the remote and the local message partition."""
import numpy as np
import pytest

from helpers import MessageCluster, OracleAdapter, create_commands, load_appendix_a5, string_docs, symbolic
from oracle.oracle import Oracle, subscription_partition
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition
from zeebe_amd.exchange import window_from_xparts

pytestmark = pytest.mark.gpu

XML = bpmn.message_catch_process()
XPART_FIELDS = [f for f in abi.XPART_DTYPE.names if f != "pad"]


class GpuAdapter:
    @staticmethod
    def deploy(p, xml):
        return p.deploy(xml)

    @staticmethod
    def intern(p, name):
        return p.intern(name)

    @staticmethod
    def intern_string(p, s):
        return p.intern_string(s)

    @staticmethod
    def window(p, cmds, docs, xparts):
        p.submit(cmds, docs, xparts)
        p.run()
        recs = p.drain()
        assert p.fallback() == [], [p.command_status(i) for i in range(len(cmds))][:4]
        return recs, p.outbox()


def clusters(P, n_inst=64, xml=XML):
    gpu = MessageCluster([Partition(partition_id=p, partition_count=P, max_instances=n_inst, max_commands=4 * n_inst,
                                    max_correlation_keys=4 * n_inst * P, max_records_per_batch=256)
                          for p in range(1, P + 1)], GpuAdapter, xml)
    orc = MessageCluster([Oracle(partition_id=p, partition_count=P) for p in range(1, P + 1)], OracleAdapter, xml)
    return gpu, orc


def assert_same_logs(gpu, orc):
    assert len(gpu.log) == len(orc.log)
    for (ph, p, gr, gob), (ph2, p2, orr, oob) in zip(gpu.log, orc.log):
        assert (ph, p) == (ph2, p2)
        assert len(gr) == len(orr), (ph, p, len(gr), len(orr))
        for f in abi.PARITY_FIELDS:
            if not np.array_equal(gr[f], orr[f]):
                bad = np.nonzero(gr[f] != orr[f])[0][:5]
                raise AssertionError("%s p%d field %s at %s: got %s want %s" % (ph, p, f, bad, gr[f][bad], orr[f][bad]))
        assert len(gob) == len(oob), (ph, p)
        for f in XPART_FIELDS:
            assert np.array_equal(gob[f], oob[f]), (ph, p, f, gob[f], oob[f])


def assert_same_state(gpu, orc):
    from oracle import statedb as SD
    for g, o in zip(gpu.parts, orc.parts):
        gs, os_ = g.state(), o.state()
        assert gs == os_, (sorted(set(gs) ^ set(os_)))[:6]
        strings = o.strings()
        assert g.state_db() == SD.encode_rows(os_, o.process_tables(), lambda i: strings[i])


@pytest.mark.parametrize("case", ["remote", "local"])
def test_gpu_appendix_a5(case):
    spec = load_appendix_a5()[case]
    P = spec["partitions"]
    gpu, orc = clusters(P, 4)
    for cl in (gpu, orc):
        kid = cl.intern_keys([spec["correlation_key"]])[0]
        outs = []
        for p in range(1, P + 1):
            if p != 1:
                outs.append(abi.make_xparts(0))
                continue
            c = create_commands(1)
            c["doc_count"] = 1
            outs.append(cl._run("create", p, c, string_docs(cl.var_id, [kid])))
        cl.exchange("subscribe", outs)
        cl.publish([kid], [subscription_partition(spec["correlation_key"], P)])
    assert_same_logs(gpu, orc)
    for (phase, p, recs, ob), step in zip(gpu.log, spec["steps"]):
        g = gpu.parts[p - 1]
        got = [t[:6] for t in symbolic(recs, g.element_id, g.name, partition=p)]
        assert got == [list(t) for t in step["batch"]], (phase, p)
    assert_same_state(gpu, orc)


@pytest.mark.parametrize("P", [1, 2, 3, 8])
def test_gpu_cluster_parity(P):
    n = 48
    gpu, orc = clusters(P, n)
    for cl in (gpu, orc):
        keys = ["k-%d-%d" % (p, i) for p in range(1, P + 1) for i in range(n)]
        ids = cl.intern_keys(keys)
        cl.create(n, [ids[(p - 1) * n:p * n] for p in range(1, P + 1)])
    assert_same_logs(gpu, orc)
    assert_same_state(gpu, orc)  # subscriptions open (PROCESS_SUBSCRIPTION OPENED, MESSAGE_SUBSCRIPTION rows)
    for cl in (gpu, orc):
        keys = ["k-%d-%d" % (p, i) for p in range(1, P + 1) for i in range(n)]
        ids = cl.intern_keys(keys)
        cl.publish(ids, [subscription_partition(k, P) for k in keys])
    assert_same_logs(gpu, orc)
    assert_same_state(gpu, orc)
    done = sum(int(np.sum((r["value_type"] == abi.VT_PROCESS_INSTANCE) & (r["intent"] == 5) & (r["element_idx"] == 0)))
               for _, _, r, _ in gpu.log)
    assert done == n * P


def test_gpu_shared_key_and_duplicate_open():
    # two instances waiting on one key: one correlation per process (lowest element instance key);
    # a duplicate MESSAGE_SUBSCRIPTION:CREATE is acknowledged and rejected
    gpu, orc = clusters(2, 8)
    for cl in (gpu, orc):
        kid = cl.intern_keys(["a"])[0]  # message partition 2
        c = create_commands(2)
        c["doc_count"] = 1
        c["doc_begin"] = [0, 1]
        ob = cl._run("create", 1, c, string_docs(cl.var_id, [kid, kid]))
        cmds, xp = window_from_xparts(np.concatenate([ob, ob[:1]]))
        cl.log.append(("dup",) + (2,) + cl.ad.window(cl.parts[1], cmds, None, xp))
        cl.exchange("subscribe", [abi.make_xparts(0), cl.log[-1][3]])
        cl.publish([kid], [2])
    assert_same_logs(gpu, orc)
    assert_same_state(gpu, orc)
    rej = [r for r in gpu.log[1][2] if r["record_type"] == abi.RT_REJECTION]
    assert len(rej) == 1
    # MessageSubscriptionCreateProcessor.SUBSCRIPTION_ALREADY_OPENED_MESSAGE
    assert gpu.parts[1].reason(rej[0]) == (
        "Expected to open a new message subscription for element with key '%d' and message name 'msg', but there "
        "is already a message subscription for that element key and message name opened" % int(rej[0]["scope_key"]))


def test_gpu_outbox_device_buckets():
    # the device outbox is bucketed by target partition and stable in log order
    P = 4
    n = 64
    gpu, _ = clusters(P, n)
    keys = ["x%d" % i for i in range(n)]
    ids = gpu.intern_keys(keys)
    c = create_commands(n)
    c["doc_count"] = 1
    c["doc_begin"] = np.arange(n)
    p1 = gpu.parts[0]
    p1.submit(c, string_docs(gpu.var_id, ids))
    p1.run()
    p1.drain()
    host = p1.outbox()
    ptr, counts = p1.outbox_device()
    assert counts.sum() == len(host)
    got = np.zeros(int(counts.sum()), dtype=abi.XPART_DTYPE)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    assert hip.hipMemcpy(got.ctypes.data, ptr, got.nbytes, 2) == 0  # hipMemcpyDeviceToHost
    want = np.concatenate([host[host["target_partition"] == t] for t in range(1, P + 1)])
    for f in XPART_FIELDS:
        assert np.array_equal(got[f], want[f]), f
    assert [int(x) for x in counts] == [int(np.sum(host["target_partition"] == t)) for t in range(1, P + 1)]


@pytest.mark.parametrize("P", [1, 4])
def test_gpu_device_exchange_runs_the_protocol(P):
    """The bench path: device-resident windows, device outbox buckets, device-to-device exchange
    between P partitions on one GPU (no host relabelling): every instance completes, the
    per-partition record/transition counts equal the oracle cluster's."""
    import torch
    from zeebe_amd.exchange import LocalExchange
    n = 512
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev).cuda_stream  # one stream shared by the partitions (exchange order)
    parts = [Partition(partition_id=p, partition_count=P, max_instances=n, max_commands=4 * n,
                       max_correlation_keys=n * P, max_records_per_batch=128, stream=stream) for p in range(1, P + 1)]
    keys = ["k-%d-%d" % (p, i) for p in range(1, P + 1) for i in range(n)]
    for part in parts:
        part.deploy(XML)
        ids = part.intern_strings(keys)
    var_id, name_id = parts[0].intern("key"), parts[0].intern("msg")
    owner = parts[0].string_partitions(ids, P)
    flags = abi.RUN_NO_RESULTS
    bufs = []
    for p, part in enumerate(parts, 1):
        c = create_commands(n)
        c["doc_count"] = 1
        c["doc_begin"] = np.arange(n)
        d = string_docs(var_id, ids[(p - 1) * n:p * n])
        tc = torch.from_numpy(c.view(np.uint8).copy()).to(dev)
        td = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
        bufs += [tc, td]
        part.submit_device(tc.data_ptr(), n, td.data_ptr(), n)
        part.run(flags)
    ex = LocalExchange(parts, 4 * n, dev)
    for _ in range(4):
        if sum(ex.step()) == 0:
            break
        ex.deliver(flags | abi.RUN_ACCUMULATE)
    for p, part in enumerate(parts, 1):
        mine = ids[owner == p]
        pub = abi.make_commands(len(mine))
        pub["instance"] = mine
        pub["kind"] = abi.CMD_PUBLISH
        pub["ref"] = name_id
        tp = torch.from_numpy(pub.view(np.uint8).copy()).to(dev)
        bufs.append(tp)
        part.submit_device(tp.data_ptr(), len(mine))
        part.run(flags | abi.RUN_ACCUMULATE)
    for _ in range(4):
        if sum(ex.step()) == 0:
            break
        ex.deliver(flags | abi.RUN_ACCUMULATE)
    torch.cuda.synchronize()
    st = [part.stats() for part in parts]
    assert all(s["fallback"] == 0 for s in st), st
    assert sum(s["completed_instances"] for s in st) == n * P
    # the oracle cluster on the same inputs
    orc = MessageCluster([Oracle(partition_id=p, partition_count=P) for p in range(1, P + 1)], OracleAdapter, XML)
    oids = orc.intern_keys(keys)
    orc.create(n, [oids[(p - 1) * n:p * n] for p in range(1, P + 1)])
    orc.publish(oids, [int(x) for x in owner])
    for s, o in zip(st, orc.parts):
        c = o.counters()
        assert s["transitions"] == c["transitions"] and s["completed_instances"] == c["completed_instances"]
    # records of every partition (device stats) = the oracle's
    assert sum(s["records"] for s in st) == sum(len(r) for _, _, r, _ in orc.log)


def _exchange_protocol(P, n, drain):
    """test_gpu_device_exchange_runs_the_protocol's device path with results: every window's drained
    records and outbox, and the final states."""
    import torch
    from zeebe_amd.exchange import LocalExchange
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev).cuda_stream
    parts = [Partition(partition_id=p, partition_count=P, max_instances=n, max_commands=4 * n,
                       max_correlation_keys=n * P, max_records_per_batch=128, stream=stream) for p in range(1, P + 1)]
    keys = ["k-%d-%d" % (p, i) for p in range(1, P + 1) for i in range(n)]
    for part in parts:
        part.deploy(XML)
        ids = part.intern_strings(keys)
    var_id, name_id = parts[0].intern("key"), parts[0].intern("msg")
    owner = parts[0].string_partitions(ids, P)
    out, bufs = [], []

    def collect(tag):
        for p, part in enumerate(parts, 1):
            if part.L.zbhip_pending_records(part.h) or tag == "create":
                out.append((tag, p, part.drain().copy(), part.outbox().copy()))

    for p, part in enumerate(parts, 1):
        c = create_commands(n)
        c["doc_count"] = 1
        c["doc_begin"] = np.arange(n)
        d = string_docs(var_id, ids[(p - 1) * n:p * n])
        tc = torch.from_numpy(c.view(np.uint8).copy()).to(dev)
        td = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
        bufs += [tc, td]
        part.submit_device(tc.data_ptr(), n, td.data_ptr(), n)
        part.run(0)
        out.append(("create", p, part.drain().copy(), part.outbox().copy()))
    ex = LocalExchange(parts, 4 * n, dev)
    for phase in ("subscribe", "publish", "correlate"):
        if phase == "publish":
            for p, part in enumerate(parts, 1):
                mine = ids[owner == p]
                pub = abi.make_commands(len(mine))
                pub["instance"] = mine
                pub["kind"] = abi.CMD_PUBLISH
                pub["ref"] = name_id
                tp = torch.from_numpy(pub.view(np.uint8).copy()).to(dev)
                bufs.append(tp)
                part.submit_device(tp.data_ptr(), len(mine))
                part.run(0)
                out.append(("publish", p, part.drain().copy(), part.outbox().copy()))
            continue
        for r in range(4):
            sizes = ex.step()
            if sum(sizes) == 0:
                break
            for t, part in enumerate(parts):
                if sizes[t]:
                    part.submit_xparts_device(ex.inbox[t].data_ptr(), sizes[t])
                    part.run(0)
                    out.append((phase, t + 1, part.drain().copy(), part.outbox().copy()))
    torch.cuda.synchronize()
    return out, [part.state() for part in parts]


def test_gpu_subject_sorted_device_windows(monkeypatch):
    # a message partition's device window launched in subject order (ZBHIP_SUBJECT_SORT): the same
    # records, outboxes and states as the window in arrival order
    monkeypatch.delenv("ZBHIP_SUBJECT_SORT", raising=False)
    base, base_state = _exchange_protocol(4, 512, True)
    monkeypatch.setenv("ZBHIP_SUBJECT_SORT", "1")
    got, got_state = _exchange_protocol(4, 512, True)
    assert len(got) == len(base)
    for (t1, p1, r1, o1), (t2, p2, r2, o2) in zip(got, base):
        assert (t1, p1) == (t2, p2)
        assert len(r1) == len(r2) and len(o1) == len(o2), (t1, p1)
        for f in abi.PARITY_FIELDS:
            assert np.array_equal(r1[f], r2[f]), (t1, p1, f)
        for f in XPART_FIELDS:
            assert np.array_equal(o1[f], o2[f]), (t1, p1, f)
    assert got_state == base_state
