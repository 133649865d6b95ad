"""Shared test helpers: golden fixtures, symbolic record tuples, workload builders."""
import json
import os

import numpy as np

from zeebe_amd import abi, bpmn

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

VT_SHORT = {abi.VT_PROCESS_INSTANCE: "PI", abi.VT_PROCESS_INSTANCE_CREATION: "PIC", abi.VT_JOB: "JOB",
            abi.VT_VARIABLE: "VAR", abi.VT_PROCESS_EVENT: "PE", abi.VT_MESSAGE: "MSG",
            abi.VT_MESSAGE_SUBSCRIPTION: "MS", abi.VT_PROCESS_MESSAGE_SUBSCRIPTION: "PMS"}
RT_SHORT = {abi.RT_EVENT: "E", abi.RT_COMMAND: "C", abi.RT_REJECTION: "R"}


def load_appendix_a():
    with open(os.path.join(GOLDEN, "appendix_a.json")) as f:
        return json.load(f)


def process_xml(spec):
    if "fixture" in spec:
        with open(os.path.join(GOLDEN, spec["fixture"])) as f:
            return f.read()
    return getattr(bpmn, spec["builder"])(**spec.get("args", {}))


def sym_key(k, partition=1):
    if k < 0:
        return -1
    p = k >> 51
    if p != partition:
        return "p%dk%d" % (p, k - (p << 51))
    return "k%d" % (k - (partition << 51))


def symbolic(records, element_id, var_name, reason=None, partition=1):
    """records: numpy RECORD_DTYPE rows; element_id(proc, elem) -> str; var_name(id) -> str;
    reason(i) -> rejection text.  Returns list of golden-style tuples."""
    out = []
    for i, r in enumerate(records):
        vt = int(r["value_type"])
        if vt == abi.VT_VARIABLE:
            el = var_name(int(r["element_idx"]))
        else:
            el = element_id(int(r["process_idx"]), int(r["element_idx"])) if r["element_idx"] >= 0 else None
        t = [RT_SHORT[int(r["record_type"])], VT_SHORT.get(vt, str(vt)), abi.intent_name(vt, int(r["intent"])),
             el, sym_key(int(r["key"]), partition), sym_key(int(r["scope_key"]), partition)]
        if int(r["record_type"]) == abi.RT_REJECTION:
            t.append(abi.REJECTION_TYPES[int(r["rejection_type"])])
            t.append(reason(i) if reason else None)
        out.append(t)
    return out


def split_batches(records):
    """Split drained records (ordered by source, ordinal) into per-source batches."""
    batches = []
    last = None
    for i, r in enumerate(records):
        if last is None or int(r["source_index"]) != last:
            batches.append([])
            last = int(r["source_index"])
        batches[-1].append(i)
    return batches


def create_commands(n, process_idx=0, first_instance=0):
    c = abi.make_commands(n)
    c["instance"] = np.arange(first_instance, first_instance + n, dtype=np.uint32)
    c["kind"] = abi.CMD_CREATE
    c["ref"] = process_idx
    return c


def complete_commands(instances, job_ordinals):
    c = abi.make_commands(len(instances))
    c["instance"] = np.asarray(instances, dtype=np.uint32)
    c["kind"] = abi.CMD_JOB_COMPLETE
    c["ref"] = np.asarray(job_ordinals, dtype=np.uint16)
    return c


def amount_docs(values, name_id, decimal=False):
    d = abi.make_docs(len(values))
    d["name_id"] = name_id
    d["type"] = abi.DOC_DEC if decimal else abi.DOC_INT
    d["value"] = np.asarray(values, dtype=np.int64)
    return d


def load_appendix_a5():
    with open(os.path.join(GOLDEN, "appendix_a5.json")) as f:
        return json.load(f)


def string_docs(name_id, string_ids):
    d = abi.make_docs(len(string_ids))
    d["name_id"] = name_id
    d["type"] = abi.DOC_STR
    d["value"] = np.asarray(string_ids, dtype=np.int64)
    return d


def publish_commands(string_ids, name_id):
    c = abi.make_commands(len(string_ids))
    c["instance"] = np.asarray(string_ids, dtype=np.uint32)
    c["kind"] = abi.CMD_PUBLISH
    c["ref"] = name_id
    return c


class MessageCluster:
    """Config 5 driver over P partitions (oracles or GPU partitions, same interface through
    `adapter`): create instances, run the subscription exchange to quiescence, publish one
    message per correlation key on its message partition, exchange again.  Every window's
    records and outbox are logged per partition in order, so two clusters fed the same inputs
    can be compared step by step."""

    def __init__(self, parts, adapter, xml, message_name="msg", var="key"):
        self.parts = parts
        self.P = len(parts)
        self.ad = adapter
        for p in parts:
            adapter.deploy(p, xml)
        self.name_id = adapter.intern(parts[0], message_name)
        self.var_id = adapter.intern(parts[0], var)
        for p in parts:
            assert adapter.intern(p, message_name) == self.name_id and adapter.intern(p, var) == self.var_id
        self.log = []  # (phase, partition, records, outbox)

    def intern_keys(self, keys):
        ids = None
        for p in self.parts:
            got = [self.ad.intern_string(p, k) for k in keys]
            assert ids is None or got == ids  # replicated dictionary
            ids = got
        return ids

    def _run(self, phase, p, cmds, docs=None, xparts=None):
        recs, ob = self.ad.window(self.parts[p - 1], cmds, docs, xparts)
        self.log.append((phase, p, recs, ob))
        return ob

    def exchange(self, phase, outboxes):
        from zeebe_amd.exchange import route, window_from_xparts
        rounds = 0
        while any(len(o) for o in outboxes):
            inbox = route(outboxes, self.P)
            outboxes = [abi.make_xparts(0) for _ in range(self.P)]
            for t in range(1, self.P + 1):
                if len(inbox[t - 1]):
                    cmds, xp = window_from_xparts(inbox[t - 1])
                    outboxes[t - 1] = self._run(phase, t, cmds, None, xp)
            rounds += 1
            assert rounds < 8
        return rounds

    def create(self, instances_per_partition, keys):
        """keys[p-1][i] = correlation key string of instance i on partition p."""
        outboxes = []
        for p in range(1, self.P + 1):
            n = instances_per_partition
            ids = keys[p - 1]
            cmds = create_commands(n)
            cmds["doc_count"] = 1
            cmds["doc_begin"] = np.arange(n, dtype=np.uint32)
            outboxes.append(self._run("create", p, cmds, string_docs(self.var_id, ids)))
        self.exchange("subscribe", outboxes)

    def commands(self, phase, cmds_per_partition):
        """One window per partition (None: none), then the exchange to quiescence."""
        outboxes = []
        for p in range(1, self.P + 1):
            c = cmds_per_partition[p - 1]
            outboxes.append(self._run(phase, p, c) if c is not None and len(c) else abi.make_xparts(0))
        self.exchange(phase, outboxes)

    def publish(self, key_ids, key_partition):
        """key_partition[i] = message partition of key_ids[i] (SubscriptionUtil)."""
        outboxes = []
        for p in range(1, self.P + 1):
            mine = [k for k, q in zip(key_ids, key_partition) if q == p]
            if mine:
                outboxes.append(self._run("publish", p, publish_commands(mine, self.name_id)))
            else:
                outboxes.append(abi.make_xparts(0))
        self.exchange("correlate", outboxes)


class OracleAdapter:
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
        p.clear_records()
        p.submit(cmds, docs, xparts)
        p.run()
        return p.records(), p.outbox()
