"""Writes tests/golden/appendix_a.json: the per-instance record sequences of the
BASELINE workloads, transcribed by hand from the reference code paths (SURVEY.md
Appendix A, each step cited there) and cross-checked against the subsequences the
reference's own tests pin (ParallelGatewayTest.java:142-233,354-401,
ExclusiveGatewayTest.java:208-251, CreateProcessInstanceTest.java:173-211).

These are written as *rules* (not produced by running the oracle): the oracle and
the GPU executor are both checked against them.

Record tuple: [recordType, valueType, intent, elementId, key, scopeKey] where keys
are symbolic "kN" = N-th key generated in the partition (encodePartitionId(1, N)),
or -1.  recordType E/C/R, valueType short names.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def one_task_batches(proc="benchmark", start="start", task="task", end="end",
                     f1="SequenceFlow_0xll35j", f2="SequenceFlow_1wkb5x5"):
    # A.1 batch 1 (CreateProcessInstanceProcessor.java:129-158, ProcessProcessor.java:55-61,
    # StartEventProcessor.java:45-67, JobWorkerTaskProcessor.java:49-61)
    b1 = [
        ["C", "PI", "ACTIVATE_ELEMENT", proc, "k1", -1],
        ["E", "PIC", "CREATED", proc, "k2", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", proc, "k1", -1],
        ["E", "PI", "ELEMENT_ACTIVATED", proc, "k1", -1],
        ["C", "PI", "ACTIVATE_ELEMENT", start, -1, "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", start, "k3", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATED", start, "k3", "k1"],
        ["C", "PI", "COMPLETE_ELEMENT", start, "k3", "k1"],
        ["E", "PI", "ELEMENT_COMPLETING", start, "k3", "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", start, "k3", "k1"],
        ["E", "PI", "SEQUENCE_FLOW_TAKEN", f1, "k4", "k1"],
        ["C", "PI", "ACTIVATE_ELEMENT", task, "k5", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", task, "k5", "k1"],
        ["E", "JOB", "CREATED", task, "k6", "k5"],
        ["E", "PI", "ELEMENT_ACTIVATED", task, "k5", "k1"],
    ]
    # A.1 batch 2 (JobCompleteProcessor.java:53-92, EventHandle.java:151-158, EndEventProcessor.java:110-134)
    b2 = [
        ["E", "JOB", "COMPLETED", task, "k6", "k5"],
        ["E", "PE", "TRIGGERING", task, "k7", "k5"],
        ["C", "PI", "COMPLETE_ELEMENT", task, "k5", "k1"],
        ["E", "PI", "ELEMENT_COMPLETING", task, "k5", "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", task, "k5", "k1"],
        ["E", "PI", "SEQUENCE_FLOW_TAKEN", f2, "k8", "k1"],
        ["C", "PI", "ACTIVATE_ELEMENT", end, "k9", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", end, "k9", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATED", end, "k9", "k1"],
        ["E", "PI", "ELEMENT_COMPLETING", end, "k9", "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", end, "k9", "k1"],
        ["C", "PI", "COMPLETE_ELEMENT", proc, "k1", -1],
        ["E", "PI", "ELEMENT_COMPLETING", proc, "k1", -1],
        ["E", "PI", "ELEMENT_COMPLETED", proc, "k1", -1],
    ]
    return b1, b2


def linear_batches(n=10, proc="linear", flows=None):
    """A.2: batch 1 as A.1 with task1; each middle completion 10 records; last as A.1 batch 2."""
    tasks = ["task%d" % i for i in range(1, n + 1)]
    b1, _ = one_task_batches(proc, "start", tasks[0], "end", flows[0], None)
    batches = [b1]
    k = 6  # last key so far (job of task1)
    task_key = 5
    for i in range(n - 1):
        job = k
        pe, sft, nxt, njob = k + 1, k + 2, k + 3, k + 4
        batches.append([
            ["E", "JOB", "COMPLETED", tasks[i], "k%d" % job, "k%d" % task_key],
            ["E", "PE", "TRIGGERING", tasks[i], "k%d" % pe, "k%d" % task_key],
            ["C", "PI", "COMPLETE_ELEMENT", tasks[i], "k%d" % task_key, "k1"],
            ["E", "PI", "ELEMENT_COMPLETING", tasks[i], "k%d" % task_key, "k1"],
            ["E", "PI", "ELEMENT_COMPLETED", tasks[i], "k%d" % task_key, "k1"],
            ["E", "PI", "SEQUENCE_FLOW_TAKEN", flows[i + 1], "k%d" % sft, "k1"],
            ["C", "PI", "ACTIVATE_ELEMENT", tasks[i + 1], "k%d" % nxt, "k1"],
            ["E", "PI", "ELEMENT_ACTIVATING", tasks[i + 1], "k%d" % nxt, "k1"],
            ["E", "JOB", "CREATED", tasks[i + 1], "k%d" % njob, "k%d" % nxt],
            ["E", "PI", "ELEMENT_ACTIVATED", tasks[i + 1], "k%d" % nxt, "k1"],
        ])
        k, task_key = njob, nxt
    job = k
    pe, sft, endk = k + 1, k + 2, k + 3
    batches.append([
        ["E", "JOB", "COMPLETED", tasks[-1], "k%d" % job, "k%d" % task_key],
        ["E", "PE", "TRIGGERING", tasks[-1], "k%d" % pe, "k%d" % task_key],
        ["C", "PI", "COMPLETE_ELEMENT", tasks[-1], "k%d" % task_key, "k1"],
        ["E", "PI", "ELEMENT_COMPLETING", tasks[-1], "k%d" % task_key, "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", tasks[-1], "k%d" % task_key, "k1"],
        ["E", "PI", "SEQUENCE_FLOW_TAKEN", flows[n], "k%d" % sft, "k1"],
        ["C", "PI", "ACTIVATE_ELEMENT", "end", "k%d" % endk, "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", "end", "k%d" % endk, "k1"],
        ["E", "PI", "ELEMENT_ACTIVATED", "end", "k%d" % endk, "k1"],
        ["E", "PI", "ELEMENT_COMPLETING", "end", "k%d" % endk, "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", "end", "k%d" % endk, "k1"],
        ["C", "PI", "COMPLETE_ELEMENT", proc, "k1", -1],
        ["E", "PI", "ELEMENT_COMPLETING", proc, "k1", -1],
        ["E", "PI", "ELEMENT_COMPLETED", proc, "k1", -1],
    ])
    return batches


def xor_batch(branch, proc="xorProcess", f_start="sequenceFlow_1"):
    """A.3 (amount present): VARIABLE:CREATED first, then one batch to process completion."""
    flow, end = ("high", "endHigh") if branch == "high" else ("low", "endLow")
    return [
        ["E", "VAR", "CREATED", "amount", "k2", "k1"],
        ["C", "PI", "ACTIVATE_ELEMENT", proc, "k1", -1],
        ["E", "PIC", "CREATED", proc, "k3", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", proc, "k1", -1],
        ["E", "PI", "ELEMENT_ACTIVATED", proc, "k1", -1],
        ["C", "PI", "ACTIVATE_ELEMENT", "start", -1, "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", "start", "k4", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATED", "start", "k4", "k1"],
        ["C", "PI", "COMPLETE_ELEMENT", "start", "k4", "k1"],
        ["E", "PI", "ELEMENT_COMPLETING", "start", "k4", "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", "start", "k4", "k1"],
        ["E", "PI", "SEQUENCE_FLOW_TAKEN", f_start, "k5", "k1"],
        ["C", "PI", "ACTIVATE_ELEMENT", "xor", "k6", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", "xor", "k6", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATED", "xor", "k6", "k1"],
        ["E", "PI", "ELEMENT_COMPLETING", "xor", "k6", "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", "xor", "k6", "k1"],
        ["E", "PI", "SEQUENCE_FLOW_TAKEN", flow, "k7", "k1"],
        ["C", "PI", "ACTIVATE_ELEMENT", end, "k8", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", end, "k8", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATED", end, "k8", "k1"],
        ["E", "PI", "ELEMENT_COMPLETING", end, "k8", "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", end, "k8", "k1"],
        ["C", "PI", "COMPLETE_ELEMENT", proc, "k1", -1],
        ["E", "PI", "ELEMENT_COMPLETING", proc, "k1", -1],
        ["E", "PI", "ELEMENT_COMPLETED", proc, "k1", -1],
    ]


def fork_join_batch(n=8, proc="forkjoin", f_start="sequenceFlow_1"):
    """A.4 straight-through: one batch; the first join activation is accepted, n-1 rejected.
    Outgoing order of the fork = reverse document order of the flows (ModelWalker.java:75-79),
    i.e. f_n .. f_1 for the builder model."""
    reason = ("Expected to be able to activate parallel gateway 'join', "
              "but not all sequence flows have been taken.")
    b = [
        ["C", "PI", "ACTIVATE_ELEMENT", proc, "k1", -1],
        ["E", "PIC", "CREATED", proc, "k2", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", proc, "k1", -1],
        ["E", "PI", "ELEMENT_ACTIVATED", proc, "k1", -1],
        ["C", "PI", "ACTIVATE_ELEMENT", "start", -1, "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", "start", "k3", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATED", "start", "k3", "k1"],
        ["C", "PI", "COMPLETE_ELEMENT", "start", "k3", "k1"],
        ["E", "PI", "ELEMENT_COMPLETING", "start", "k3", "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", "start", "k3", "k1"],
        ["E", "PI", "SEQUENCE_FLOW_TAKEN", f_start, "k4", "k1"],
        ["C", "PI", "ACTIVATE_ELEMENT", "fork", "k5", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", "fork", "k5", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATED", "fork", "k5", "k1"],
        ["E", "PI", "ELEMENT_COMPLETING", "fork", "k5", "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", "fork", "k5", "k1"],
    ]
    k = 5
    join_keys = []
    for i in range(n, 0, -1):
        b.append(["E", "PI", "SEQUENCE_FLOW_TAKEN", "f%d" % i, "k%d" % (k + 1), "k1"])
        b.append(["C", "PI", "ACTIVATE_ELEMENT", "join", "k%d" % (k + 2), "k1"])
        join_keys.append(k + 2)
        k += 2
    jk = join_keys[0]
    b += [
        ["E", "PI", "ELEMENT_ACTIVATING", "join", "k%d" % jk, "k1"],
        ["E", "PI", "ELEMENT_ACTIVATED", "join", "k%d" % jk, "k1"],
        ["E", "PI", "ELEMENT_COMPLETING", "join", "k%d" % jk, "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", "join", "k%d" % jk, "k1"],
        ["E", "PI", "SEQUENCE_FLOW_TAKEN", "toEnd", "k%d" % (k + 1), "k1"],
        ["C", "PI", "ACTIVATE_ELEMENT", "end", "k%d" % (k + 2), "k1"],
    ]
    endk = k + 2
    for rk in join_keys[1:]:
        b.append(["R", "PI", "ACTIVATE_ELEMENT", "join", "k%d" % rk, "k1", "INVALID_STATE", reason])
    b += [
        ["E", "PI", "ELEMENT_ACTIVATING", "end", "k%d" % endk, "k1"],
        ["E", "PI", "ELEMENT_ACTIVATED", "end", "k%d" % endk, "k1"],
        ["E", "PI", "ELEMENT_COMPLETING", "end", "k%d" % endk, "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", "end", "k%d" % endk, "k1"],
        ["C", "PI", "COMPLETE_ELEMENT", proc, "k1", -1],
        ["E", "PI", "ELEMENT_COMPLETING", proc, "k1", -1],
        ["E", "PI", "ELEMENT_COMPLETED", proc, "k1", -1],
    ]
    return b


def main():
    cases = {
        "one_task": {"process": {"fixture": "one_task.bpmn"}, "batches": list(one_task_batches())},
        "linear10": {"process": {"builder": "linear_process", "args": {"n_tasks": 10}},
                     "batches": linear_batches(10, "linear",
                                               ["sequenceFlow_%d" % i for i in range(1, 12)])},
        "xor_high": {"process": {"builder": "xor_process"}, "amount": 1500, "batches": [xor_batch("high")]},
        "xor_low": {"process": {"builder": "xor_process"}, "amount": 1000, "batches": [xor_batch("low")]},
        "fork_join8": {"process": {"builder": "fork_join_process", "args": {"branches": 8}},
                       "batches": [fork_join_batch(8)]},
    }
    with open(os.path.join(HERE, "appendix_a.json"), "w") as f:
        json.dump(cases, f, indent=1)


if __name__ == "__main__":
    main()
