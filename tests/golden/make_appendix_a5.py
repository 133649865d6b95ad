"""Writes tests/golden/appendix_a5.json: SURVEY.md Appendix A.5 (message catch event correlated
across partitions, config 5) as per-partition, per-batch record sequences, transcribed by hand
from the reference code paths:

* IntermediateCatchEventProcessor.onActivate -> CatchEventBehavior.subscribeToMessageEvent
  (processing/common/CatchEventBehavior.java:248-283): ACTIVATING, PROCESS_MESSAGE_SUBSCRIPTION
  CREATING (+key), [local: C MESSAGE_SUBSCRIPTION:CREATE], ACTIVATED;
* SubscriptionCommandSender.handleFollowUpCommandBasedOnPartition (:304-320): same partition ->
  follow-up command (key -1) processed in the same batch, else a post-commit send;
* MessageSubscriptionCreateProcessor (:83-104): CREATED (+key), ack PROCESS_MESSAGE_SUBSCRIPTION:CREATE;
* ProcessMessageSubscriptionCreateProcessor: CREATED (subscription key);
* MessagePublishProcessor.handleNewMessage: PUBLISHED (+key), CORRELATING per subscription,
  PROCESS_MESSAGE_SUBSCRIPTION:CORRELATE sends, EXPIRED (time-to-live 0);
* ProcessMessageSubscriptionCorrelateProcessor: CORRELATED, EventHandle.activateElement
  (PROCESS_EVENT:TRIGGERING +key, C COMPLETE_ELEMENT), ack MESSAGE_SUBSCRIPTION:CORRELATE;
* MessageSubscriptionCorrelateProcessor: CORRELATED (subscription key).

The partition of a correlation key is SubscriptionUtil.getSubscriptionPartitionId; "a" goes to
partition 2 of 2 (SubscriptionUtilTest: hash("a") = 97).  Keys: "kN" = N-th key of the record's
own partition, "pPkN" = a key of partition P (a foreign key inside the record value).

Tuple: [recordType, valueType, intent, elementId, key, scopeKey (PI: flowScopeKey; PMS/MS:
elementInstanceKey)].
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def start_part(eik_scope="k1"):
    return [
        ["E", "VAR", "CREATED", "key", "k2", "k1"],
        ["C", "PI", "ACTIVATE_ELEMENT", "process", "k1", -1],
        ["E", "PIC", "CREATED", "process", "k3", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", "process", "k1", -1],
        ["E", "PI", "ELEMENT_ACTIVATED", "process", "k1", -1],
        ["C", "PI", "ACTIVATE_ELEMENT", "start", -1, "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", "start", "k4", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATED", "start", "k4", "k1"],
        ["C", "PI", "COMPLETE_ELEMENT", "start", "k4", "k1"],
        ["E", "PI", "ELEMENT_COMPLETING", "start", "k4", "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", "start", "k4", "k1"],
        ["E", "PI", "SEQUENCE_FLOW_TAKEN", "sequenceFlow_1", "k5", "k1"],
        ["C", "PI", "ACTIVATE_ELEMENT", "catch", "k6", "k1"],
        ["E", "PI", "ELEMENT_ACTIVATING", "catch", "k6", "k1"],
        ["E", "PMS", "CREATING", "catch", "k7", "k6"],
    ]


def end_part(sft, end):
    return [
        ["E", "PI", "ELEMENT_COMPLETING", "catch", "k6", "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", "catch", "k6", "k1"],
        ["E", "PI", "SEQUENCE_FLOW_TAKEN", "sequenceFlow_2", sft, "k1"],
        ["C", "PI", "ACTIVATE_ELEMENT", "end", end, "k1"],
    ]


def end_tail(end):
    return [
        ["E", "PI", "ELEMENT_ACTIVATING", "end", end, "k1"],
        ["E", "PI", "ELEMENT_ACTIVATED", "end", end, "k1"],
        ["E", "PI", "ELEMENT_COMPLETING", "end", end, "k1"],
        ["E", "PI", "ELEMENT_COMPLETED", "end", end, "k1"],
        ["C", "PI", "COMPLETE_ELEMENT", "process", "k1", -1],
        ["E", "PI", "ELEMENT_COMPLETING", "process", "k1", -1],
        ["E", "PI", "ELEMENT_COMPLETED", "process", "k1", -1],
    ]


def remote():
    """PI partition 1, message partition 2 (correlation key "a")."""
    return {
        "partitions": 2, "correlation_key": "a",
        "steps": [
            {"phase": "create", "partition": 1, "batch": start_part() + [
                ["E", "PI", "ELEMENT_ACTIVATED", "catch", "k6", "k1"]],
             "outbox": [["MSG_SUB_CREATE", 2]]},
            {"phase": "open", "partition": 2, "batch": [
                ["E", "MS", "CREATED", None, "k1", "p1k6"]],
             "outbox": [["PMS_CREATE", 1]]},
            {"phase": "opened", "partition": 1, "batch": [
                ["E", "PMS", "CREATED", "catch", "k7", "k6"]],
             "outbox": []},
            {"phase": "publish", "partition": 2, "batch": [
                ["E", "MSG", "PUBLISHED", None, "k2", -1],
                ["E", "MS", "CORRELATING", None, "k1", "p1k6"],
                ["E", "MSG", "EXPIRED", None, "k2", -1]],
             "outbox": [["PMS_CORRELATE", 1]]},
            {"phase": "correlate", "partition": 1, "batch": [
                ["E", "PMS", "CORRELATED", "catch", "k7", "k6"],
                ["E", "PE", "TRIGGERING", "catch", "k8", "k6"],
                ["C", "PI", "COMPLETE_ELEMENT", "catch", "k6", "k1"]] + end_part("k9", "k10") + end_tail("k10"),
             "outbox": [["MSG_SUB_CORRELATE", 2]]},
            {"phase": "ack", "partition": 2, "batch": [
                ["E", "MS", "CORRELATED", None, "k1", "p1k6"]],
             "outbox": []},
        ],
    }


def local():
    """One partition: every subscription command is a follow-up command of the same batch."""
    return {
        "partitions": 1, "correlation_key": "k-0",
        "steps": [
            {"phase": "create", "partition": 1, "batch": start_part() + [
                ["C", "MS", "CREATE", None, -1, "k6"],
                ["E", "PI", "ELEMENT_ACTIVATED", "catch", "k6", "k1"],
                ["E", "MS", "CREATED", None, "k8", "k6"],
                ["C", "PMS", "CREATE", None, -1, "k6"],
                ["E", "PMS", "CREATED", "catch", "k7", "k6"]],
             "outbox": []},
            {"phase": "publish", "partition": 1, "batch": [
                ["E", "MSG", "PUBLISHED", None, "k9", -1],
                ["E", "MS", "CORRELATING", None, "k8", "k6"],
                ["C", "PMS", "CORRELATE", None, -1, "k6"],
                ["E", "MSG", "EXPIRED", None, "k9", -1],
                ["E", "PMS", "CORRELATED", "catch", "k7", "k6"],
                ["E", "PE", "TRIGGERING", "catch", "k10", "k6"],
                ["C", "PI", "COMPLETE_ELEMENT", "catch", "k6", "k1"],
                ["C", "MS", "CORRELATE", None, -1, "k6"]] + end_part("k11", "k12") + [
                ["E", "MS", "CORRELATED", None, "k8", "k6"]] + end_tail("k12"),
             "outbox": []},
        ],
    }


if __name__ == "__main__":
    with open(os.path.join(HERE, "appendix_a5.json"), "w") as f:
        json.dump({"remote": remote(), "local": local()}, f, indent=1)
