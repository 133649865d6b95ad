"""Shared test helpers: golden fixtures, symbolic record tuples, workload builders."""
import json
import os

import numpy as np

from zeebe_amd import abi, bpmn

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

VT_SHORT = {abi.VT_PROCESS_INSTANCE: "PI", abi.VT_PROCESS_INSTANCE_CREATION: "PIC", abi.VT_JOB: "JOB",
            abi.VT_VARIABLE: "VAR", abi.VT_PROCESS_EVENT: "PE"}
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
