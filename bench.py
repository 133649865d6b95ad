"""Headline benchmark: BPMN element transitions/s (+ completed instances/s) of the MI355X
batch executor on BASELINE.json configs[1] -- a linear 10-service-task process, 10^6
instances per GPU, jobs auto-completed in 10 phases (one JOB:COMPLETE window per task).

One step = one full pass of that workload over the partition: a window of 10^6
PROCESS_INSTANCE_CREATION:CREATE commands followed by 10 windows of 10^6 JOB:COMPLETE,
each processed to quiescence (63 transitions, 119 records per instance).  Inputs are
synthetic and already resident in HBM; nothing is skipped inside the timed region.

Multi-GPU: one process per GPU, one Zeebe partition per GPU (Protocol.encodePartitionId),
instances keyed to partitions; no data-path collective (weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config linear10|one_task|xor|forkjoin8|boundary10|msg]

--config msg is configs[4]: a message catch event correlated across partitions (one partition per
GPU; the subscription commands between partitions go through RCCL all-to-all over xGMI, or, with
--virtual-partitions P on one GPU, through device-to-device copies between P partitions).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SURVEY_BYTES_PER_TRANSITION = {"linear10": 114.4, "one_task": 100.4, "xor": 93.3, "forkjoin8": 92.8,
                               "forkjoin8_tasks": 92.8}


def workload(name):
    from zeebe_amd import bpmn
    if name == "linear10":
        return bpmn.linear_process(10), 1_000_000, 10, False
    if name == "one_task":
        with open(os.path.join(ROOT, "tests", "golden", "one_task.bpmn")) as f:
            return f.read(), 1_000_000, 1, False
    if name == "xor":
        return bpmn.xor_process(), 10_000_000, 0, True
    if name == "forkjoin8":
        return bpmn.fork_join_process(8), 10_000_000, 0, False
    if name == "forkjoin8_tasks":  # variant 4b: a service task per branch, jobs completed in random branch order
        return bpmn.fork_join_process(8, tasks=True), 10_000_000, 8, False
    if name == "boundary10":  # linear-10 with an interrupting timer boundary event on every task (KScope)
        b = bpmn.createExecutableProcess("boundary10").startEvent("start")
        for i in range(10):
            b.serviceTask("task%d" % i, "benchmark-task").boundaryEvent("late%d" % i).timerWithDuration("PT1H")
            b.endEvent("lateEnd%d" % i).moveToActivity("task%d" % i)
        return b.endEvent("end").done(), 1_000_000, 10, False
    raise SystemExit("unknown config " + name)


# first job key ordinal and ordinals per phase of the JOB:COMPLETE windows (kernels.hip key order:
# per task SFT, ACTIVATE, [the boundary's timer,] job; per completion PROCESS_EVENT + those)
JOB_ORDINALS = {"boundary10": (6, 5)}
# forkjoin8_tasks records per window (SURVEY App. A.4 variant 4b): CREATE 63 (start, fork, 8 x
# [SFT, ACTIVATE, ACTIVATING, JOB:CREATED, ACTIVATED]); completions 1..7 9 each (JOB:COMPLETED,
# PROCESS_EVENT, COMPLETE, COMPLETING, COMPLETED, SFT, ACTIVATE(join), the join's rejection... )
FJ8T_RECORDS = None  # measured by the bench's probe (records of one instance per window)


def algorithmic_bytes(name, n, phases):
    """Minimum HBM bytes of the k_step launches of one step ('Bytes per unit'):
    commands read (16 B), compact records written (8 B), per-command header written (8 B),
    instance header read+written (16+16 B), element-instance slots read/written (8 B each),
    variables (16 B) and join counters (16 B) where the workload has them."""
    if name in ("linear10", "one_task"):
        # CREATE: cmd 16 + hdr 32 + 15 recs*8 + hdr 8 + 1 slot write 8
        b = 16 + 32 + 15 * 8 + 8 + 8
        for p in range(phases):
            last = p == phases - 1
            recs = 14 if last else 10
            # JOB:COMPLETE: cmd 16 + hdr 32 + slot read 8 (+ write 8 if another task follows) + recs + hdr 8
            b += 16 + 32 + 8 + (0 if last else 8) + recs * 8 + 8
        return b * n
    if name == "xor":
        return (16 + 16 + 32 + 26 * 8 + 8) * n  # + the amount document entry (16 B)
    if name == "forkjoin8":
        return (16 + 32 + 52 * 8 + 8) * n
    if name == "forkjoin8_tasks":
        # CREATE: cmd 16 + hdr 32 + records (start .. 8 branches activated, 8 jobs) + hdr 8 + 8 slots
        # written (8 B each) + join words 16; each JOB:COMPLETE: cmd 16 + hdr 32 + the 8 slots read
        # (the lane loads the instance's table) + the remaining ones written + join words read and
        # written 32 + records + hdr 8.  Records per window: see records_forkjoin8_tasks
        recs = FJ8T_RECORDS
        b = 16 + 32 + recs[0] * 8 + 8 + 8 * 8 + 16
        for p in range(phases):
            left = 8 - p - 1
            b += 16 + 32 + (8 - p) * 8 + left * 8 + 32 + recs[p + 1] * 8 + 8
        return b * n
    if name == "boundary10":
        # linear-10's rows plus the timer: CREATE 16 records + the timer row written (16 B); each
        # JOB:COMPLETE 12 records (TIMER:CANCELED, the next TIMER:CREATED), the timer row read and
        # written, the canceled dueDate (8 B); the last one 15 records
        b = 16 + 32 + 16 * 8 + 8 + 8 + 16
        for p in range(phases):
            last = p == phases - 1
            b += 16 + 32 + 8 + (0 if last else 8) + (15 if last else 12) * 8 + 8 + 16 + 16 + 8
        return b * n
    return 0


def run_msg(args, world, rank, local_rank, dist):
    """configs[4]: start -> message catch (`= key`) -> end, n instances per partition, one message per
    correlation key published on its message partition (SubscriptionUtil), time-to-live 0.  One step:
    CREATE windows -> exchange (MESSAGE_SUBSCRIPTION:CREATE, PROCESS_MESSAGE_SUBSCRIPTION:CREATE) ->
    PUBLISH windows -> exchange (PROCESS_MESSAGE_SUBSCRIPTION:CORRELATE, MESSAGE_SUBSCRIPTION:CORRELATE),
    every window run to quiescence on the device; inputs resident in HBM."""
    import numpy as np
    import torch

    from zeebe_amd import abi, bpmn
    from zeebe_amd.engine import Partition
    from zeebe_amd.exchange import XPART_BYTES, DeviceExchange, LocalExchange

    dev = torch.device("cuda", local_rank)
    vp = args.virtual_partitions if world == 1 else 1
    P = world * vp  # partitions in the cluster
    n = args.instances or 1_000_000
    stream = torch.cuda.Stream(device=dev).cuda_stream  # one stream shared by the partitions (exchange order)
    my_parts = list(range(rank * vp + 1, rank * vp + vp + 1))
    parts = [Partition(partition_id=p, partition_count=P, device=local_rank, max_instances=n, max_commands=4 * n,
                       max_correlation_keys=n * P, max_records_per_batch=128, stream=stream,
                       trusted_device_windows=True) for p in my_parts]
    xml = bpmn.message_catch_process()
    t_setup = time.perf_counter()
    blob_parts, offs = [], [0]
    for p in range(1, P + 1):
        for i in range(n):
            b = b"k-%d-%d" % (p, i)
            blob_parts.append(b)
            offs.append(offs[-1] + len(b))
    blob = b"".join(blob_parts)
    offsets = np.asarray(offs, dtype=np.uint64)
    import ctypes as C
    ids = None
    for part in parts:
        part.deploy(xml)
        got = np.zeros(n * P, dtype=np.uint32)
        from zeebe_amd.native import check
        check(part.L.zbhip_intern_strings(part.h, blob, offsets.ctypes.data, n * P, got.ctypes.data))
        assert ids is None or np.array_equal(ids, got)  # replicated dictionary
        ids = got
    var_id, name_id = parts[0].intern("key"), parts[0].intern("msg")
    owner = parts[0].string_partitions(ids, P)  # message partition of every key
    windows = []
    for p, part in zip(my_parts, parts):
        create = abi.make_commands(n)
        create["instance"] = np.arange(n, dtype=np.uint32)
        create["kind"] = abi.CMD_CREATE
        create["doc_count"] = 1
        create["doc_begin"] = np.arange(n, dtype=np.uint32)
        docs = abi.make_docs(n)
        docs["name_id"] = var_id
        docs["type"] = abi.DOC_STR
        docs["value"] = ids[(p - 1) * n:p * n]
        mine = ids[owner == p]
        pub = abi.make_commands(len(mine))
        pub["instance"] = mine
        pub["kind"] = abi.CMD_PUBLISH
        pub["ref"] = name_id
        windows.append(tuple(torch.from_numpy(a.view(np.uint8).copy()).to(dev) for a in (create, docs, pub)) +
                       (len(mine),))
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup
    exch = LocalExchange(parts, 4 * n, dev) if world == 1 else DeviceExchange(max_entries=4 * n, device=dev)
    staging = torch.empty(4 * n * XPART_BYTES, dtype=torch.uint8, device=dev) if world > 1 else None

    def exchange_until_quiet(flags):
        rounds = 0
        while rounds < 6:
            if world == 1:
                if sum(exch.step()) == 0:
                    break
                exch.deliver(flags)
            else:
                _, total = exch.exchange_partition(parts[0], staging, flags)
                if total == 0:
                    break
            rounds += 1
        return rounds

    def step(first, timed=False):
        flags = abi.RUN_NO_RESULTS | (abi.RUN_TIMED if timed else 0)
        for k, (part, (cw, dw, pw, npub)) in enumerate(zip(parts, windows)):
            part.submit_device(cw.data_ptr(), n, dw.data_ptr(), n)
            part.run(flags | (0 if first else abi.RUN_ACCUMULATE))
        r1 = exchange_until_quiet(flags | abi.RUN_ACCUMULATE)
        for part, (cw, dw, pw, npub) in zip(parts, windows):
            part.submit_device(pw.data_ptr(), npub)
            part.run(flags | abi.RUN_ACCUMULATE)
        r2 = exchange_until_quiet(flags | abi.RUN_ACCUMULATE)
        return r1, r2

    for k in range(args.warmup):
        step(first=(k == 0))
    for part in parts:
        s = part.stats()
        assert s["fallback"] == 0, s
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rounds = None
    for k in range(args.steps):
        rounds = step(first=(k == 0))
    st = [part.stats() for part in parts]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    assert all(s["fallback"] == 0 for s in st), st
    tr = sum(s["transitions"] for s in st)
    comp = sum(s["completed_instances"] for s in st)
    recs = sum(s["records"] for s in st)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor([tr, comp, recs], dtype=torch.float64, device=dev)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        tr, comp, recs = (int(x) for x in c.tolist())
    assert comp == n * P * args.steps, (comp, n * P * args.steps)
    # device time of the lifecycle kernel launches + key scans (untimed pass)
    step(first=True, timed=True)
    st = [part.stats() for part in parts]
    dev_ms = sum(s["step_ms"] for s in st)
    # bytes per instance over both partitions: commands 16 B x 4 windows,
    # records 8 B x rows, instance rows 16+8+16 B read+written per PI window, slot rows 48 B written
    # and read, 48-byte subscription commands written, bucketed, exchanged and read (x4)
    rows = sum(s["records"] for s in st) / max(1, n * P)
    alg_per_inst = 16 * 6 + 8 * (rows + 6 * 10) + 2 * 40 * 3 + 2 * 48 * 3 + 4 * 48 * 4
    alg = alg_per_inst * n * P
    # HBM traffic per step of the config-5 kernels (k_step, key scan, bucketing) from the PMC passes
    # of this build (scripts/evidence.sh: pmc_traffic.py "zb::" <steps>); null without a summary
    traffic, traffic_src = None, None
    tpath = os.path.join(ROOT, "profiles", "pmc_%s.json" % ("msg" if vp == 1 else "msg%d" % vp))
    if os.path.exists(tpath) and not args.instances and world == 1:
        with open(tpath) as f:
            traffic = json.load(f).get("traffic_bytes_per_step")
        traffic_src = os.path.relpath(tpath, ROOT)
    result = {
        "metric": "BPMN element transitions/sec + completed instances/sec, 1/2/4/8 MI355X",
        "value": tr / elapsed,
        "unit": "transitions/s",
        "completed_instances_per_s": comp / elapsed,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic: %d instances/partition, correlation keys k-<p>-<i>, one message per key (TTL 0)" % n,
        "config": {"workload": "configs[4] message catch event correlated across partitions",
                   "instances_per_partition": n, "partitions": P, "partitions_per_gpu": vp,
                   "exchange": "rccl all_to_all_single" if world > 1 else ("device copies" if P > 1 else "none (local)"),
                   "exchange_rounds": rounds, "parallelism": "one partition per GPU (dp%d)" % world},
        "records_per_s": recs / elapsed,
        "setup_s": setup_s,
        "roofline": {"bound": "hbm", "kernel": "k_step<KMsg> + key scan", "achieved": alg / (dev_ms * 1e-3) / 1e9 / world,
                     "peak": PEAK_HBM_GBPS, "unit": "GB/s", "frac": alg / (dev_ms * 1e-3) / 1e9 / world / PEAK_HBM_GBPS,
                     "traffic": traffic, "traffic_unit": "bytes/step (all zb:: kernels)", "traffic_source": traffic_src,
                     "algorithmic_bytes_per_step": alg, "algorithmic_bytes_per_instance": alg_per_inst,
                     "device_ms_per_step": dev_ms},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.oracle import bench_msg
        th = args.cpu_threads
        n_cpu = max(1000, args.cpu_instances // 6)
        sec, ctr, ccomp = bench_msg(xml, th, n_cpu)
        result["cpu_baseline"] = {"value": ctr / sec, "unit": "transitions/s", "cores": th, "kind": "port",
                                  "completed_instances_per_s": ccomp / sec,
                                  "sample": "%d partitions (1 per thread) x %d instances, cross-partition exchange "
                                            "between phases on the calling thread, %.1f s" % (th, n_cpu, sec)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def host_io_pass(args, xml, n, host_windows, local_rank, recs_per_batch):
    """The boundary as a host adapter uses it (zbhip_submit from host memory, zbhip_run with results,
    zbhip_drain into host memory): every window crosses PCIe in (16 B per command) and out (the
    compact records), and the host expands them to 80-byte zbhip_record with keys relabelled in
    DbKeyGenerator order.  A fresh partition; one untimed pass, then one timed pass.  Never `value`."""
    import time

    from zeebe_amd import abi
    from zeebe_amd.engine import Partition

    part = Partition(partition_id=1, partition_count=1, device=local_rank, max_instances=n, max_commands=n,
                     max_records_per_batch=recs_per_batch)
    part.deploy(xml)
    if host_windows[0][1] is not None:
        part.intern("amount")
    res = None
    for timed in (False, True):
        t0 = time.perf_counter()
        recs = trans = 0
        buf = None  # one record buffer for the pass (Partition.drain reuses it)
        split = [0.0, 0.0, 0.0]  # submit / run (+ results copy and relabel bookkeeping) / drain
        for w, (cmds, docs) in enumerate(host_windows):
            ta = time.perf_counter()
            part.submit(cmds, docs)
            tb = time.perf_counter()
            part.run(abi.RUN_ACCUMULATE if w else 0)  # statistics summed over the pass's windows
            tc = time.perf_counter()
            out = part.drain(buf)
            base = out.base if out.base is not None else out
            if buf is None or len(base) > len(buf):
                buf = base
            split[0] += tb - ta
            split[1] += tc - tb
            split[2] += time.perf_counter() - tc
            recs += len(out)
        sec = time.perf_counter() - t0
        trans = part.stats()["transitions"]
        if timed:
            res = {"value": trans / sec, "unit": "transitions/s", "records_per_s": recs / sec,
                   "ms_per_step": sec * 1e3, "records_per_step": recs,
                   "submit_ms": split[0] * 1e3, "run_ms": split[1] * 1e3, "drain_ms": split[2] * 1e3,
                   "path": "zbhip_submit (host buffers) + zbhip_run + zbhip_drain (80-B records, relabelled keys)"}
    res["log_bytes"] = log_device_pass(xml, n, host_windows, local_rank, recs_per_batch)
    return res


def log_device_pass(xml, n, host_windows, local_rank, recs_per_batch):
    """Submit -> log bytes: the same windows from host buffers, run with the records left in HBM
    (ZBHIP_RUN_DEVICE_RECORDS) and serialised there (zbhip_serialize_log_device: the reference's
    log entries, keys relabelled on the device); then once more with the bytes copied to host memory
    (PCIe-inclusive).  A fresh partition; one untimed pass, then the timed passes."""
    import ctypes as C
    import time

    import numpy as np

    from zeebe_amd import abi
    from zeebe_amd.engine import Partition

    part = Partition(partition_id=1, partition_count=1, device=local_rank, max_instances=n, max_commands=n,
                     max_records_per_batch=recs_per_batch)
    part.deploy(xml)
    if host_windows[0][1] is not None:
        part.intern("amount")
    pos = [np.arange(len(c), dtype=np.int64) * 2 + 1 for c, _ in host_windows]
    host_buf = None
    res = {}
    # 'host': zbhip_log_copy_async -- window k's bytes cross PCIe into the handle's pinned buffer while window
    # k+1 is submitted, run and serialised (the wait for copy k is the 'copy' time); 'host_sync': the
    # synchronous zbhip_log_device_copy into pageable memory (round 5's path)
    for mode in ("warm", "hbm", "host", "host_sync"):
        t0 = time.perf_counter()
        total = 0
        split = [0.0, 0.0, 0.0, 0.0]  # submit / run / serialise / copy
        first = 1
        pending = None
        for w, (cmds, docs) in enumerate(host_windows):
            ta = time.perf_counter()
            part.submit(cmds, docs)
            tb = time.perf_counter()
            part.run(abi.RUN_DEVICE_RECORDS | (abi.RUN_ACCUMULATE if w else 0))
            tc = time.perf_counter()
            ptr, used = part.serialize_log_device(pos[w], first, 1700000000123, copy=False)
            td = time.perf_counter()
            if mode == "host_sync":
                if host_buf is None or len(host_buf) < used:
                    host_buf = C.create_string_buffer(int(used * 1.25) + 1)
                part.L.zbhip_log_device_copy(part.h, host_buf, used)
            elif mode in ("host", "warm"):
                landing = part.log_copy_async(used)
                if pending is not None:
                    part.log_copy_wait(pending)  # window k-1's log bytes are in host memory
                pending = landing
            te = time.perf_counter()
            first += int(part.L.zbhip_pending_records(part.h))
            total += used
            for k, dt in enumerate((tb - ta, tc - tb, td - tc, te - td)):
                split[k] += dt
        if pending is not None:
            te = time.perf_counter()
            part.log_copy_wait(pending)
            split[3] += time.perf_counter() - te
        sec = time.perf_counter() - t0
        if mode != "warm":
            trans = part.stats()["transitions"]
            res[mode] = {"value": trans / sec, "unit": "transitions/s", "log_bytes_per_step": total,
                         "log_GBps": total / sec / 1e9, "ms_per_step": sec * 1e3, "submit_ms": split[0] * 1e3,
                         "run_ms": split[1] * 1e3, "serialize_ms": split[2] * 1e3, "copy_ms": split[3] * 1e3}
    res["path"] = ("zbhip_submit (host buffers) + zbhip_run(DEVICE_RECORDS) + zbhip_serialize_log_device "
                   "(log entries in HBM); 'host' adds zbhip_log_copy_async into the handle's pinned host buffers "
                   "(double-buffered, overlapping the next window), 'host_sync' zbhip_log_device_copy into "
                   "pageable memory")
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="linear10")
    ap.add_argument("--instances", type=int, default=0, help="override instances per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--untrusted-windows", action="store_true",
                    help="check every device window's subjects on the device (k_subject_check) in the timed loop")
    ap.add_argument("--no-templates", action="store_true",
                    help="general path only: CREATE batch templates off (ZBHIP_NO_TEMPLATES)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-instances", type=int, default=300_000, help="instances per CPU thread (bounded sample)")
    ap.add_argument("--host-io", action="store_true",
                    help="time the host-boundary passes (host command buffers and drained records; log bytes in "
                         "HBM and copied to the host) -- on by default for the N = 1 linear10 run, never `value`")
    ap.add_argument("--no-host-io", action="store_true", help="skip the host-boundary passes")
    ap.add_argument("--virtual-partitions", type=int, default=1,
                    help="--config msg on one GPU: partitions hosted by this process (exchange by device copies)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `bench.py --gpus N` without a launcher: start one rank per GPU (spawned interpreters; this
        # process never touches the GPU) and exit with the ranks' status
        import torch.multiprocessing as mp
        port = _free_port()
        ctx = mp.start_processes(_spawned_rank, args=(args.gpus, port, sys.argv[1:]), nprocs=args.gpus,
                                 join=True, start_method="spawn")
        return ctx
    run_rank(args)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawned_rank(rank, world, port, argv):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.argv = [sys.argv[0]] + list(argv)
    main()


def probe_fork_join_tasks(xml, local_rank):
    """One instance of variant 4b in results mode: the key ordinal of each branch's job (JOB:CREATED
    of task t<b> in the CREATE batch) and the records of each window (CREATE, then 8 completions)."""
    import numpy as np
    from zeebe_amd import abi
    from zeebe_amd.engine import Partition
    part = Partition(max_instances=1, max_commands=1, max_records_per_batch=64, device=local_rank)
    part.deploy(xml)
    c = abi.make_commands(1)
    c["kind"] = abi.CMD_CREATE
    part.submit(c)
    part.run()
    recs = part.drain()
    counts = [len(recs)]
    ids = part.processes[0].element_ids
    ords = np.zeros(8, dtype=np.uint16)
    for r in recs:
        if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED:
            ords[int(ids[int(r["element_idx"])][1:]) - 1] = part.resolve_key(int(r["key"]))[1]
    for b in range(8):
        c = abi.make_commands(1)
        c["kind"], c["ref"] = abi.CMD_JOB_COMPLETE, ords[b]
        part.submit(c)
        part.run()
        counts.append(len(part.drain()))
    part.close()
    return ords, counts


def run_rank(args):
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        # one partition per GPU: the ranks the launcher started are the GPUs measured
        assert dist.get_world_size() == world and (args.gpus in (1, world)), (dist.get_world_size(), args.gpus)
    torch.cuda.set_device(local_rank)
    if args.config == "msg":
        return run_msg(args, world, rank, local_rank, dist)

    from zeebe_amd import abi
    from zeebe_amd.engine import Partition

    if args.no_templates:
        os.environ["ZBHIP_NO_TEMPLATES"] = "1"  # read by zbhip_run at every launch
    xml, n, phases, with_amount = workload(args.config)
    if args.instances:
        n = args.instances
    recs_per_batch = 64
    # the partition launches on a torch stream, so torch.cuda.Event brackets its kernels directly
    pstream = torch.cuda.Stream(device=torch.device("cuda", local_rank))
    part = Partition(partition_id=rank + 1, partition_count=world, device=local_rank, max_instances=n,
                     max_commands=n, max_records_per_batch=recs_per_batch, stream=pstream.cuda_stream,
                     # one command per instance per window, by construction; --untrusted-windows runs the
                     # device subject check (k_subject_check) on every window as an untrusted caller would
                     trusted_device_windows=not args.untrusted_windows)
    part.deploy(xml)
    name = part.intern("amount") if with_amount else None

    # ---- synthetic windows, built once and kept resident in HBM ----
    dev = torch.device("cuda", local_rank)
    windows = []
    host_windows = []  # the same windows as host buffers, for the PCIe-inclusive pass (--host-io)
    create = abi.make_commands(n)
    create["instance"] = np.arange(n, dtype=np.uint32)
    create["kind"] = abi.CMD_CREATE
    docs_t = None
    if with_amount:
        rng = np.random.default_rng(0x5EED03 + rank)
        docs = abi.make_docs(n)
        docs["name_id"] = name
        docs["type"] = abi.DOC_INT
        docs["value"] = rng.integers(0, 2001, n)
        create["doc_count"] = 1
        create["doc_begin"] = np.arange(n, dtype=np.uint32)
        docs_t = torch.from_numpy(docs.view(np.uint8).copy()).to(dev)
    windows.append(torch.from_numpy(create.view(np.uint8).copy()).to(dev))
    host_windows.append((create, docs if with_amount else None))
    job_ord, per_phase = JOB_ORDINALS.get(args.config, (5 if not with_amount else 6, 4))
    branch_ord = None
    if args.config == "forkjoin8_tasks":
        # variant 4b: every instance completes its 8 branch jobs in its own seeded random order
        # (seed 0x5EED04); the job key ordinals and records per window come from a probe
        branch_ord, recs = probe_fork_join_tasks(xml, local_rank)
        global FJ8T_RECORDS
        FJ8T_RECORDS = recs
        rng = np.random.default_rng(0x5EED04 + rank)
        order = np.argsort(rng.random((n, 8)), axis=1).astype(np.uint16)  # a permutation per instance
    for p in range(phases):
        c = abi.make_commands(n)
        c["instance"] = np.arange(n, dtype=np.uint32)
        c["kind"] = abi.CMD_JOB_COMPLETE
        c["ref"] = job_ord + per_phase * p if branch_ord is None else branch_ord[order[:, p]]
        windows.append(torch.from_numpy(c.view(np.uint8).copy()).to(dev))
        host_windows.append((c, None))
    torch.cuda.synchronize()

    def step(first, timed=False):
        """One pass over the workload: every window is enqueued back to back on the partition's
        stream (no host wait between windows); statistics accumulate on the device."""
        for i, w in enumerate(windows):
            if i == 0 and docs_t is not None:
                part.submit_device(w.data_ptr(), n, docs_t.data_ptr(), n)
            else:
                part.submit_device(w.data_ptr(), n)
            flags = abi.RUN_NO_RESULTS | (abi.RUN_TIMED if timed else 0)
            if not (first and i == 0):
                flags |= abi.RUN_ACCUMULATE
            part.run(flags)

    for k in range(args.warmup):
        step(first=(k == 0))
    s = part.stats()
    assert s["fallback"] == 0, s
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(pstream)
    for k in range(args.steps):
        step(first=(k == 0))
    ev1.record(pstream)
    s = part.stats()  # waits for the partition's stream
    tpl_timed = s["template_batches"]
    torch.cuda.synchronize()
    span_ms = ev0.elapsed_time(ev1)  # device time of the timed region: the k_step launches back to back
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    assert s["fallback"] == 0, s
    tot_tr, tot_comp, tot_recs = s["transitions"], s["completed_instances"], s["records"]
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor([tot_tr, tot_comp, tot_recs], dtype=torch.float64, device=dev)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        tot_tr, tot_comp, tot_recs = (int(x) for x in c.tolist())

    # ---- kernel timing with HIP events on the partition's stream ----
    # k_step_avg_ms: events around the whole timed region / launches -- the kernels run back to back
    # (the host enqueues faster than they execute), so this is the kernel duration plus the small
    # inter-kernel gap, i.e. conservative against rocprofv3's per-kernel average.  The event-pair
    # figure (events around every launch in a separate pass) is reported too; its per-launch event
    # commands inflate it.
    launches = len(windows)
    k_step_avg_ms = span_ms / (args.steps * launches)
    step(first=True, timed=True)
    s = part.stats()
    tr, step_ms = s["transitions"], s["step_ms"]
    alg = algorithmic_bytes(args.config, n, phases)
    achieved = alg / launches / (k_step_avg_ms * 1e-3) / 1e9
    survey_bpt = SURVEY_BYTES_PER_TRANSITION.get(args.config)
    # HBM traffic per launch from the PMC passes of this build (scripts/pmc.sh + scripts/pmc_traffic.py,
    # FETCH_SIZE x2 gfx950 correction); null when no summary for this workload is committed
    traffic, traffic_src = None, None
    tpath = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
    if os.path.exists(tpath) and not args.instances:
        with open(tpath) as f:
            traffic = json.load(f)["traffic_bytes_per_launch"]
        traffic_src = os.path.relpath(tpath, ROOT)

    result = {
        "metric": "BPMN element transitions/sec + completed instances/sec, 1/2/4/8 MI355X",
        "value": tot_tr / elapsed,
        "unit": "transitions/s",
        "completed_instances_per_s": tot_comp / elapsed,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic: %d instances/GPU, jobs auto-completed in %d phases, inputs resident in HBM" % (n, phases),
        "config": {"workload": {"linear10": "configs[1] linear 10-service-task process, 1M instances, auto-completed jobs",
                                "one_task": "configs[0] one_task.bpmn create->job complete",
                                "xor": "configs[2] exclusive gateway `= amount > 1000`, 10M instances",
                                "forkjoin8": "configs[3] parallel fork/join 8 branches, 10M instances",
                                "forkjoin8_tasks": "configs[3] variant 4b: fork/join 8 branches with a service task "
                                                   "each, jobs completed in random branch order, 10M instances",
                                "boundary10": "linear 10 service tasks, each with an interrupting timer boundary "
                                              "event (timers created and canceled), 1M instances"}[args.config],
                   "instances_per_gpu": n, "windows_per_step": len(windows), "partitions": world,
                   "parallelism": "one partition per GPU (dp%d)" % world, "max_commands_in_batch": 100,
                   "templates": not args.no_templates, "subject_check": bool(args.untrusted_windows)},
        "records_per_s": tot_recs / elapsed,
        # CREATE batches copied from a template the general path recorded (kernels.hip tpl_create)
        "template_batches_per_step": tpl_timed / max(1, args.steps),
        "roofline": {"bound": "hbm", "kernel": "k_step", "achieved": achieved, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBPS, "traffic": traffic, "traffic_unit": "bytes/launch",
                     "traffic_source": traffic_src, "algorithmic_bytes_per_launch": alg / launches,
                     "algorithmic_bytes_per_step": alg,
                     "bytes_per_transition": alg / max(tr, 1),
                     "k_step_avg_ms": k_step_avg_ms, "k_step_timing": "HIP events over the timed region / launches",
                     "k_step_event_pairs_ms": step_ms / launches,
                     "compaction": "fused into k_step (wavefront scan)",
                     "survey_bytes_per_transition": survey_bpt,
                     "survey_model_GBps": (tr / (k_step_avg_ms * launches * 1e-3) * survey_bpt / 1e9) if survey_bpt else None},
    }
    # the end-to-end figures a host adapter sees (submit from host memory -> records or log bytes), timed
    # by the default run too (N = 1, the headline config linear10; ~6 s): reported beside `value`, never
    # as it (other configs only with --host-io: their drained records outgrow host memory)
    if (args.host_io or (world == 1 and not args.no_host_io and args.config == "linear10")) and rank == 0:
        result["host_io"] = host_io_pass(args, xml, n, host_windows, local_rank, recs_per_batch)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.oracle import bench as cpu_bench, bench_jobs
        th = args.cpu_threads
        if branch_ord is not None:
            sec, ctr, ccomp = bench_jobs(xml, th, args.cpu_instances, branch_ord)
        else:
            sec, ctr, ccomp = cpu_bench(xml, th, args.cpu_instances, phases, with_amount)
        result["cpu_baseline"] = {"value": ctr / sec, "unit": "transitions/s", "cores": th, "kind": "port",
                                  "completed_instances_per_s": ccomp / sec,
                                  "sample": "%d partitions (1 per thread) x %d instances, same workload, %.1f s"
                                            % (th, args.cpu_instances, sec)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
