/*
 * zbhip.h — C ABI of libzbhip.so, the MI355X batch executor for Zeebe's BPMN
 * element-lifecycle hot path.
 *
 * The library replaces, for one partition, everything from
 * `Engine.process` (engine/src/main/java/io/camunda/zeebe/engine/Engine.java:99-131)
 * down to the zb-db column-family mutations, for the supported element subset
 * (process, embedded sub-process, none start/end event, service task, undefined
 * and manual task, none intermediate throw event, message intermediate catch
 * event, exclusive gateway, parallel gateway).  It is meant to sit behind the stream-platform `RecordProcessor`
 * API (stream-platform/src/main/java/io/camunda/zeebe/stream/api/RecordProcessor.java:17-108):
 * a Java host adapter buffers a window of hot-path commands from the log,
 * submits them, runs them to quiescence and re-emits the drained records per
 * source command through `ProcessingResultBuilder`.
 *
 * Conventions:
 *  - a handle is one partition; every call on one handle is single-threaded
 *    (mirrors the partition actor); different handles may run concurrently;
 *  - errors are negative ZBHIP_E* codes, nothing throws across the ABI;
 *  - device memory is owned by the handle, host buffers by the caller;
 *  - keys are generated on the device as per-instance ordinals and relabelled
 *    by zbhip_drain to the reference's keys, `Protocol.encodePartitionId(p, n)`
 *    (protocol/src/main/java/io/camunda/zeebe/protocol/Protocol.java:98-100),
 *    n advancing in submission (log) order exactly as `DbKeyGenerator.nextKey`
 *    (stream-platform/.../state/DbKeyGenerator.java:39-42) would.
 *
 * Element indexing (shared contract with the CPU oracle): element index 0 is
 * the process itself; the flow nodes and sequence flows follow in XML document
 * pre-order (an embedded sub-process, then its children, then its next sibling).
 */
#ifndef ZBHIP_H
#define ZBHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZBHIP_ABI_VERSION 11 /* 3: zbhip_element.flow_scope, start_event (embedded sub-processes);
                               4: timer boundary events (start_event / flow_source / job_retries of job
                                  workers and boundary events), zbhip_set_clock, TIMER / JOB:CANCELED /
                                  PROCESS_EVENT:TRIGGERED records, zbhip_record.partition = repetitions;
                               5: ZBHIP_OPEN_DEFER_CONTINUATIONS / ZBHIP_CMD_CONTINUE,
                                  zbhip_continuations, zbhip_pending_continuations, zbhip_current_key,
                                  zbhip_set_key_if_higher;
                               6: multi-instance bodies (ZBHIP_EL_MULTI_INSTANCE_BODY elements,
                                  ZBHIP_OP_ITEM collections), PROCESS_INSTANCE_BATCH records, VARIABLE
                                  records with inline values (ZBHIP_AUX_INLINE), six variables per
                                  activated job;
                               7: INCIDENT:CREATED records of exclusive gateways (ZBHIP_VT_INCIDENT,
                                  zbhip_incident_message), zbhip_process_csr.cond_text;
                               8: zbhip_outbox_command, zbhip_drain_command on message partitions,
                                  zeebe:ioMapping (zbhip_process_csr.mappings);
                               9: interrupting message boundary events, ZBHIP_CMD_MSG_SUB_DELETE /
                                  ZBHIP_CMD_PMS_DELETE and the DELETING / DELETE / DELETED records;
                              10: static zeebe:taskHeaders (zbhip_process_csr.header_begin /
                                  header_bytes);
                              11: multi-entry variable documents (zbhip_doc_merge_order: the merge
                                  order in zbhip_doc_entry.pad) */

/* ---- error codes ------------------------------------------------------- */
#define ZBHIP_OK 0
#define ZBHIP_EINVAL -1     /* bad argument */
#define ZBHIP_ENOMEM -2     /* capacity exhausted (instances, records, documents) */
#define ZBHIP_EDEVICE -3    /* HIP runtime error */
#define ZBHIP_EPARSE -4     /* BPMN/FEEL outside the supported subset */
#define ZBHIP_EUNSUPP -5    /* construct outside the supported subset */
#define ZBHIP_ESTATE -6     /* call out of order (e.g. drain before run) */
#define ZBHIP_ENODEV -7     /* no usable gfx950 device */

/* ---- protocol enums (protocol/src/main/resources/protocol.xml:23-72) ---- */
enum zbhip_record_type { ZBHIP_RT_EVENT = 0, ZBHIP_RT_COMMAND = 1, ZBHIP_RT_REJECTION = 2 };
enum zbhip_value_type {
  ZBHIP_VT_JOB = 0,
  ZBHIP_VT_PROCESS_INSTANCE = 5,
  ZBHIP_VT_INCIDENT = 6,
  ZBHIP_VT_MESSAGE = 10,
  ZBHIP_VT_MESSAGE_SUBSCRIPTION = 11,
  ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION = 12,
  ZBHIP_VT_MESSAGE_START_EVENT_SUBSCRIPTION = 16,  /* engine-only: message start events stay with the CPU engine */
  ZBHIP_VT_VARIABLE = 17,
  ZBHIP_VT_PROCESS_INSTANCE_CREATION = 19,
  ZBHIP_VT_PROCESS_EVENT = 24,
  ZBHIP_VT_TIMER = 15,
  ZBHIP_VT_PROCESS_INSTANCE_BATCH = 34,
  ZBHIP_VT_JOB_BATCH = 14  /* JOB_BATCH (protocol.xml:31): a job stream's push */
};
enum zbhip_rejection_type {
  ZBHIP_REJ_INVALID_ARGUMENT = 0,
  ZBHIP_REJ_NOT_FOUND = 1,
  ZBHIP_REJ_ALREADY_EXISTS = 2,
  ZBHIP_REJ_INVALID_STATE = 3,
  ZBHIP_REJ_PROCESSING_ERROR = 4,
  ZBHIP_REJ_NONE = 255
};
/* ProcessInstanceIntent (protocol/.../intent/ProcessInstanceIntent.java:22-35) */
enum zbhip_pi_intent {
  ZBHIP_PI_SEQUENCE_FLOW_TAKEN = 1,
  ZBHIP_PI_ELEMENT_ACTIVATING = 2,
  ZBHIP_PI_ELEMENT_ACTIVATED = 3,
  ZBHIP_PI_ELEMENT_COMPLETING = 4,
  ZBHIP_PI_ELEMENT_COMPLETED = 5,
  ZBHIP_PI_ELEMENT_TERMINATING = 6,
  ZBHIP_PI_ELEMENT_TERMINATED = 7,
  ZBHIP_PI_ACTIVATE_ELEMENT = 8,
  ZBHIP_PI_COMPLETE_ELEMENT = 9,
  ZBHIP_PI_TERMINATE_ELEMENT = 10
};
/* JobIntent CREATED=0 COMPLETE=1 COMPLETED=2 CANCELED=10 (JobIntent.java:19-45); VariableIntent
 * CREATED=0 UPDATED=1; ProcessEventIntent TRIGGERING=0 TRIGGERED=1; ProcessInstanceCreationIntent
 * CREATE=0 CREATED=1 */
enum { ZBHIP_JOB_CREATED = 0, ZBHIP_JOB_COMPLETE = 1, ZBHIP_JOB_COMPLETED = 2, ZBHIP_JOB_TIME_OUT = 3,
       ZBHIP_JOB_TIMED_OUT = 4, ZBHIP_JOB_FAIL = 5, ZBHIP_JOB_FAILED = 6, ZBHIP_JOB_CANCELED = 10,
       ZBHIP_JOB_THROW_ERROR = 11, ZBHIP_JOB_ERROR_THROWN = 12 };
enum { ZBHIP_JOB_BATCH_ACTIVATE = 0, ZBHIP_JOB_BATCH_ACTIVATED = 1 };  /* JobBatchIntent */
enum { ZBHIP_VAR_CREATED = 0, ZBHIP_VAR_UPDATED = 1 };
enum { ZBHIP_PE_TRIGGERING = 0, ZBHIP_PE_TRIGGERED = 1 };
enum { ZBHIP_PIC_CREATE = 0, ZBHIP_PIC_CREATED = 1 };
/* TimerIntent (protocol/.../intent/TimerIntent.java:19-30) */
enum { ZBHIP_TIMER_CREATED = 0, ZBHIP_TIMER_TRIGGER = 1, ZBHIP_TIMER_TRIGGERED = 2, ZBHIP_TIMER_CANCELED = 4 };
/* IncidentIntent CREATED=0 RESOLVE=1 RESOLVED=2 (protocol/.../intent/IncidentIntent.java:19-22) */
enum { ZBHIP_INCIDENT_CREATED = 0 };
/* ErrorType ordinals (protocol/.../record/value/ErrorType.java) of the device's incidents */
enum { ZBHIP_ERR_JOB_NO_RETRIES = 2, ZBHIP_ERR_CONDITION_ERROR = 3, ZBHIP_ERR_EXTRACT_VALUE_ERROR = 4,
       ZBHIP_ERR_UNHANDLED_ERROR_EVENT = 6 };
/* the type of a condition's non-boolean result (ResultType names in the incident message) */
enum { ZBHIP_FEEL_NULL = 0, ZBHIP_FEEL_NUMBER = 1, ZBHIP_FEEL_STRING = 2 };
/* ProcessInstanceBatchIntent (protocol/.../intent/ProcessInstanceBatchIntent.java:18-20) */
enum { ZBHIP_PIB_TERMINATE = 0, ZBHIP_PIB_ACTIVATE = 1 };
/* MessageIntent, MessageSubscriptionIntent, ProcessMessageSubscriptionIntent
 * (protocol/.../intent/MessageIntent.java:19-23, MessageSubscriptionIntent.java:19-30,
 * ProcessMessageSubscriptionIntent.java:19-28) */
enum { ZBHIP_MSG_PUBLISH = 0, ZBHIP_MSG_PUBLISHED = 1, ZBHIP_MSG_EXPIRE = 2, ZBHIP_MSG_EXPIRED = 3 };
enum { ZBHIP_MS_CREATE = 0, ZBHIP_MS_CREATED = 1, ZBHIP_MS_CORRELATE = 2, ZBHIP_MS_CORRELATED = 3,
       ZBHIP_MS_REJECT = 4, ZBHIP_MS_REJECTED = 5, ZBHIP_MS_DELETE = 6, ZBHIP_MS_DELETED = 7,
       ZBHIP_MS_CORRELATING = 8 };
enum { ZBHIP_PMS_CREATING = 0, ZBHIP_PMS_CREATE = 1, ZBHIP_PMS_CREATED = 2, ZBHIP_PMS_CORRELATE = 3,
       ZBHIP_PMS_CORRELATED = 4, ZBHIP_PMS_DELETING = 5, ZBHIP_PMS_DELETE = 6, ZBHIP_PMS_DELETED = 7 };
/* MessageStartEventSubscriptionIntent (protocol/.../intent/MessageStartEventSubscriptionIntent.java:19-21) */
enum { ZBHIP_MSES_CREATED = 0, ZBHIP_MSES_CORRELATED = 1, ZBHIP_MSES_DELETED = 2 };

/* BpmnElementType / BpmnEventType ordinals (protocol/.../value/BpmnElementType.java:24-58,
 * BpmnEventType.java:24-35) */
enum zbhip_element_type {
  ZBHIP_EL_UNSPECIFIED = 0,
  ZBHIP_EL_PROCESS = 1,
  ZBHIP_EL_SUB_PROCESS = 2,
  ZBHIP_EL_EVENT_SUB_PROCESS = 3,
  ZBHIP_EL_START_EVENT = 4,
  ZBHIP_EL_INTERMEDIATE_CATCH_EVENT = 5,
  ZBHIP_EL_INTERMEDIATE_THROW_EVENT = 6,
  ZBHIP_EL_BOUNDARY_EVENT = 7,
  ZBHIP_EL_END_EVENT = 8,
  ZBHIP_EL_SERVICE_TASK = 9,
  ZBHIP_EL_RECEIVE_TASK = 10,
  ZBHIP_EL_USER_TASK = 11,
  ZBHIP_EL_MANUAL_TASK = 12,
  ZBHIP_EL_TASK = 13,
  ZBHIP_EL_EXCLUSIVE_GATEWAY = 14,
  ZBHIP_EL_PARALLEL_GATEWAY = 15,
  ZBHIP_EL_EVENT_BASED_GATEWAY = 16,
  ZBHIP_EL_INCLUSIVE_GATEWAY = 17,
  ZBHIP_EL_SEQUENCE_FLOW = 18,
  ZBHIP_EL_MULTI_INSTANCE_BODY = 19,
  ZBHIP_EL_CALL_ACTIVITY = 20,
  ZBHIP_EL_BUSINESS_RULE_TASK = 21,
  ZBHIP_EL_SCRIPT_TASK = 22,
  ZBHIP_EL_SEND_TASK = 23
};
/* job worker tasks (BpmnElementProcessors.java:46-60 -> JobWorkerTaskProcessor): service and send
 * tasks, script / business-rule tasks with a zeebe:taskDefinition (no zeebe:script /
 * zeebe:calledDecision) */
#define ZBHIP_IS_JOB_WORKER(t) ((t) == ZBHIP_EL_SERVICE_TASK || (t) == ZBHIP_EL_SEND_TASK || \
                                (t) == ZBHIP_EL_SCRIPT_TASK || (t) == ZBHIP_EL_BUSINESS_RULE_TASK)
enum zbhip_event_type {
  ZBHIP_EV_UNSPECIFIED = 0,
  ZBHIP_EV_CONDITIONAL = 1,
  ZBHIP_EV_ERROR = 2,
  ZBHIP_EV_ESCALATION = 3,
  ZBHIP_EV_LINK = 4,
  ZBHIP_EV_MESSAGE = 5,
  ZBHIP_EV_NONE = 6,
  ZBHIP_EV_SIGNAL = 7,
  ZBHIP_EV_TERMINATE = 8,
  ZBHIP_EV_TIMER = 9
};

/* ---- compiled process (deploy-time CSR tables) -------- */
#define ZBHIP_NONE16 0xFFFFu

typedef struct zbhip_element {
  uint8_t element_type;  /* zbhip_element_type */
  uint8_t event_type;    /* zbhip_event_type */
  uint16_t out_begin;    /* outgoing flows: out_flow[out_begin .. out_begin+out_count) in getOutgoing() order */
  uint16_t out_count;
  uint16_t in_count;     /* incoming arity (parallel-gateway join arity) */
  uint16_t flow_source;  /* sequence flow: source node; boundary event: the activity it is attached to
                          * (attachedToRef, ExecutableActivity.attach); else ZBHIP_NONE16 */
  uint16_t flow_target;  /* sequence flow: target node; else ZBHIP_NONE16 */
  uint16_t condition;    /* sequence flow: condition index; ZBHIP_NONE16 = no condition;
                          * multi-instance body: the index of its inputCollection (ZBHIP_OP_ITEM
                          * instructions, one per item, or ZBHIP_OP_COLLECTION; then ZBHIP_OP_OUTPUT,
                          * then ZBHIP_OP_END) */
  uint16_t default_flow; /* exclusive gateway: default flow element; multi-instance body: the condition
                          * index of its completionCondition; sub-process: its (timer) boundary event;
                          * else ZBHIP_NONE16 */
  uint16_t job_type;     /* service task: string-table index of the job type */
  uint16_t job_retries;  /* service task: static retries; boundary event: bit 0 interrupting (cancelActivity),
                          * bits 8..15 the timer's repetitions (1 a duration, n of "Rn/", 255 "R/" infinite);
                          * multi-instance body: bit 0 isSequential */
  uint16_t join_slot;    /* sequence flow into a parallel gateway: its taken-counter slot; else NONE */
  uint16_t id;           /* string-table index of the element id */
  uint16_t message_name; /* message catch event: string-table index of the static message name;
                          * multi-instance body: string-table index of its inputElement; else NONE */
  uint16_t correlation_var; /* message catch event: string-table index of the variable of `= var` */
  uint16_t flow_scope;   /* the element's container: 0 = the process, else the embedded sub-process
                          * element (ExecutableFlowElement.getFlowScope, FlowElementInstantiationTransformer)
                          * or the multi-instance body of an inner activity (MultiInstanceActivityTransformer) */
  uint16_t start_event;  /* process / embedded sub-process: its none start event
                          * (ExecutableFlowElementContainer.getNoneStartEvent); job worker task: its
                          * (one, timer) boundary event; multi-instance body: its inner activity
                          * (ExecutableMultiInstanceBody.getInnerActivity), which shares its id; else
                          * ZBHIP_NONE16 */
  uint32_t duration_ms;  /* timer catch / boundary event: the static timeDuration in ms (Interval.parse); else 0 */
} zbhip_element;

/* FEEL condition bytecode (subset of feel-scala 1.17.0 boolean expressions,
 * SURVEY §8a row 16).  Stack machine over {NUMBER(scaled int64), BOOLEAN, NULL}. */
enum zbhip_op {
  ZBHIP_OP_END = 0,
  ZBHIP_OP_PUSH_VAR = 1,   /* arg = variable-name id */
  ZBHIP_OP_PUSH_NUM = 2,   /* literal = value * 10^ZBHIP_DEC_SCALE */
  ZBHIP_OP_PUSH_BOOL = 3,  /* arg = 0/1 */
  ZBHIP_OP_PUSH_NULL = 4,
  ZBHIP_OP_LT = 5, ZBHIP_OP_LE = 6, ZBHIP_OP_GT = 7, ZBHIP_OP_GE = 8,
  ZBHIP_OP_EQ = 9, ZBHIP_OP_NE = 10,
  ZBHIP_OP_AND = 11, ZBHIP_OP_OR = 12, ZBHIP_OP_NOT = 13,
  /* an inputCollection item: arg = its zbhip_doc_type -- INT, BOOL, NIL or STR; literal = the value (STR:
   * string-table index; zbhip_deploy interns it into the value dictionary) */
  ZBHIP_OP_ITEM = 14,
  /* a multi-instance body's inputCollection `= name`: arg = the list variable's string-table index (a
   * ZBHIP_DOC_LIST value; anything else is an incident, outside the device subset) */
  ZBHIP_OP_COLLECTION = 15,
  /* its outputCollection: arg = the collection's string-table index, literal = the outputElement
   * variable's (`= name`); a completionCondition is a condition of its own, its index in the body's
   * default_flow */
  ZBHIP_OP_OUTPUT = 16
};
#define ZBHIP_DEC_SCALE 6   /* fixed decimal scale of NUMBER values on the device */

typedef struct zbhip_insn {
  uint8_t op;
  uint8_t pad[3];
  uint32_t arg;
  int64_t literal;
} zbhip_insn;

/* A zeebe:ioMapping entry of a job worker task or an embedded sub-process in the device subset
 * (VariableMappingTransformer, deployment/model/transformer/VariableMappingTransformer.java:73-200;
 * applied by BpmnVariableMappingBehavior.java:53-156): at most one input and one output mapping per
 * element (several entries make a multi-entry document, iterated in agrona order: unpinned), a plain
 * target name, a source that is a variable reference (`= x`) or a literal (`= 5`, `= true`, `= null`,
 * `= "s"`, or a static string without '=').  Not on multi-instance inner activities. */
#define ZBHIP_MAP_VARIABLE 0xFF
typedef struct zbhip_mapping {
  uint16_t element;      /* the element the mapping belongs to */
  uint8_t output;        /* 0: input mapping (on activation), 1: output mapping (on completion) */
  uint8_t source_type;   /* ZBHIP_MAP_VARIABLE, or the zbhip_doc_type of a literal (NIL, BOOL, INT, STR) */
  uint16_t source;       /* a variable reference's name / a string literal's text: string index */
  uint16_t target;       /* the target variable's name: string index */
  int64_t literal;       /* BOOL / INT literal */
} zbhip_mapping;

typedef struct zbhip_process_csr {
  uint32_t n_elements;           /* elements[0] is the process */
  const zbhip_element* elements;
  uint32_t n_out;
  const uint16_t* out_flow;      /* CSR targets of out_begin/out_count */
  uint32_t n_conditions;
  const uint32_t* cond_begin;    /* condition c: code[cond_begin[c] .. cond_begin[c+1]) */
  uint32_t n_code;
  const zbhip_insn* code;
  uint32_t n_strings;
  const char* const* strings;    /* ids, job types, variable names (NUL-terminated) */
  uint16_t none_start;           /* element index of the none start event (NONE = none) */
  uint16_t n_join_slots;         /* taken-sequence-flow counters per instance */
  int64_t process_definition_key;
  int32_t version;
  uint16_t bpmn_process_id;      /* string index */
  uint16_t pad;
  const char* const* cond_text;  /* condition c's FEEL text after '=' (ParsedExpression.text: the incident
                                    message); "" for a multi-instance collection */
  uint32_t n_mappings;           /* zeebe:ioMapping entries (ABI 8) */
  const zbhip_mapping* mappings;
  /* zeebe:taskHeaders (ABI 10): job worker element e's customHeaders -- the msgpack map
   * BpmnJobBehavior.encodeHeaders (BpmnJobBehavior.java:219-248,365-399) writes, its entries in the
   * iteration order of the Java HashMap it builds -- at header_bytes[header_begin[e] ..
   * header_begin[e + 1]); an empty range is JobRecord.NO_HEADERS (an empty map).  NULL: no headers. */
  const uint32_t* header_begin;  /* n_elements + 1 offsets */
  const uint8_t* header_bytes;
} zbhip_process_csr;

/* Host-side compiler: BPMN XML -> CSR (engine/.../deployment/model/transformation/BpmnTransformer.java:109-127).
 * Returns ZBHIP_OK or ZBHIP_EPARSE/ZBHIP_EUNSUPP with a message in err. */
int zbhip_compile_bpmn(const char* xml, size_t len, int64_t process_definition_key, int32_t version,
                       zbhip_process_csr** out, char* err, size_t err_cap);
void zbhip_free_csr(zbhip_process_csr* csr);

/* ---- partition handle -------------------------------------------------- */
typedef struct zbhip_config {
  int32_t partition_id;          /* 1-based, as in Zeebe */
  int32_t partition_count;
  int32_t device;                /* HIP device ordinal */
  int32_t max_commands_in_batch; /* StreamProcessorContext.DEFAULT_MAX_COMMANDS_IN_BATCH = 100 */
  uint32_t max_instances;        /* instance slots in HBM */
  uint32_t max_commands;         /* commands per submitted window */
  uint32_t max_records_per_batch;/* record slots per command (0 = derive from deployed processes) */
  uint32_t max_doc_entries;      /* variable-document entries per window */
  int64_t initial_key;           /* last key already generated in the partition (0 = fresh) */
  uint32_t max_correlation_keys; /* correlation slots of this message partition (0 = no messages) */
  uint32_t flags;                /* ZBHIP_OPEN_* */
  void* stream;                  /* hipStream_t to launch on (NULL = handle-owned stream) */
} zbhip_config;

/* The caller guarantees that a device-resident window (zbhip_submit_device*) addresses every subject
 * at most once; without this flag every device window's subjects are checked on the device first. */
#define ZBHIP_OPEN_TRUSTED_DEVICE_WINDOWS 1u
/* Follow-up commands written to the log unprocessed (past maxCommandsInBatch) are not run after
 * their window: each waits as a continuation until the log reader submits it at its own log
 * position (ZBHIP_CMD_CONTINUE), so commands the log holds between the two -- other hot-path
 * commands, the CPU engine's -- come first, as in the reference.  Without the flag zbhip_run runs
 * them right after the window (a log that holds nothing in between: the benches, the oracle's
 * window model). */
#define ZBHIP_OPEN_DEFER_CONTINUATIONS 2u

typedef struct zbhip_handle zbhip_handle;

int zbhip_open(const zbhip_config* cfg, zbhip_handle** out);
void zbhip_close(zbhip_handle* h);
int zbhip_deploy(zbhip_handle* h, const zbhip_process_csr* csr, uint32_t* process_idx_out);
/* Interns a variable name for this partition; returns its id (>=0) or an error. */
int zbhip_intern(zbhip_handle* h, const char* name);
const char* zbhip_string(zbhip_handle* h, uint32_t process_idx, uint32_t string_idx);
const char* zbhip_name(zbhip_handle* h, uint32_t name_id);

/* ---- commands ------------------------------------------------------------ */
enum zbhip_command_kind {
  ZBHIP_CMD_CREATE = 1,        /* PROCESS_INSTANCE_CREATION:CREATE (CreateProcessInstanceProcessor.java:129-158) */
  ZBHIP_CMD_JOB_COMPLETE = 2,  /* JOB:COMPLETE (JobCompleteProcessor.java:47-92) */
  /* MESSAGE:PUBLISH with timeToLive 0, no messageId and no variables (MessagePublishProcessor.java
   * handleNewMessage): instance = correlation-key string id (the correlation slot of this message
   * partition), ref = message-name id (zbhip_intern).  Other publishes belong to the CPU engine. */
  ZBHIP_CMD_PUBLISH = 3,
  /* Cross-partition subscription commands (SubscriptionCommandSender.java:54-338) received from
   * another partition's outbox: doc_begin = index into the window's zbhip_xpart_cmd array.
   * instance = the command's subject: the PI instance slot (xpart.instance) for
   * PROCESS_MESSAGE_SUBSCRIPTION commands, the correlation slot (xpart.correlation_key) for
   * MESSAGE_SUBSCRIPTION commands. */
  ZBHIP_CMD_MSG_SUB_CREATE = 4,    /* MessageSubscriptionCreateProcessor.java:83-104 */
  ZBHIP_CMD_PMS_CREATE = 5,        /* ProcessMessageSubscriptionCreateProcessor */
  ZBHIP_CMD_PMS_CORRELATE = 6,     /* ProcessMessageSubscriptionCorrelateProcessor */
  ZBHIP_CMD_MSG_SUB_CORRELATE = 7, /* MessageSubscriptionCorrelateProcessor */
  /* TIMER:TRIGGER (TriggerTimerProcessor.java:81-114, written by DueDateTimerChecker for a due
   * timer): instance = the instance slot, ref = the timer key's ordinal in the instance,
   * (doc_begin | pad << 32) = the timer's dueDate (the command's TimerRecord.dueDate) */
  ZBHIP_CMD_TIMER_TRIGGER = 8,
  /* A follow-up command an earlier batch wrote to the log unprocessed (past maxCommandsInBatch,
   * ProcessingStateMachine.java:388-417) and the platform now reads back as a batch of its own, on a
   * handle opened with ZBHIP_OPEN_DEFER_CONTINUATIONS: instance = its instance slot,
   * doc_begin | pad << 32 = its continuation id (zbhip_continuations).  Host windows only. */
  ZBHIP_CMD_CONTINUE = 9,
  /* Closing a subscription (CatchEventBehavior.unsubscribeFromMessageEvent, :407-432): the
   * subscription partition's MessageSubscriptionDeleteProcessor.java:50-68 and the acknowledgement's
   * ProcessMessageSubscriptionDeleteProcessor.java:39-56; subjects as for the other subscription
   * commands (ABI 9) */
  ZBHIP_CMD_MSG_SUB_DELETE = 10,
  ZBHIP_CMD_PMS_DELETE = 11
};

/* STR values are string ids of the partition's value dictionary (zbhip_intern_string). */
/* ZBHIP_DOC_LIST: a list of scalar items (a msgpack array), value = its id in the handle's list
 * dictionary (zbhip_intern_list) -- a multi-instance inputCollection variable, an outputCollection */
enum zbhip_doc_type { ZBHIP_DOC_NIL = 0, ZBHIP_DOC_BOOL = 1, ZBHIP_DOC_INT = 2, ZBHIP_DOC_DEC = 3,
                      ZBHIP_DOC_OTHER = 4, ZBHIP_DOC_STR = 5, ZBHIP_DOC_LIST = 6 };

/* One entry of a variable document (a msgpack map entry on the reference side).
 * DEC values are value * 10^ZBHIP_DEC_SCALE (exact decimal).
 * A document of several entries (in document order) carries the order the reference merges them in:
 * IndexedDocument (state/variable/IndexedDocument.java:20-63) iterates an agrona Int2IntHashMap keyed by
 * each key's byte offset in the msgpack map.  zbhip_doc_merge_order writes it into the pad bytes: pad[0]
 * of entry i = the document index of the i-th entry iterated, pad[1] bit 0 of entry 0 = an entry sits off
 * its home slot (a removal during the iteration may then reorder the rest).  A multi-entry document
 * without a valid order, with a repeated name or with more than ZBHIP_DOC_MAX_ENTRIES entries is outside
 * the device subset (its command falls back). */
typedef struct zbhip_doc_entry {
  uint32_t name_id;
  uint8_t type;
  uint8_t pad[3];
  int64_t value;
} zbhip_doc_entry;
#define ZBHIP_DOC_MAX_ENTRIES 8

/* The merge order of a document of n entries whose keys start at the byte offsets key_offsets[0..n)
 * (strictly increasing: the offsets in the caller's msgpack bytes of the document) into entries[0..n)'s
 * pad bytes, as above: the agrona 1.19.2 Int2IntHashMap (initial capacity 8, load factor 0.65,
 * evenHash, linear probing by pairs, doubling past the threshold) IndexedDocument.index fills, iterated
 * from the top slot (or from below the first free slot when the top one is taken) downwards.
 * ZBHIP_EINVAL for unordered offsets or n > 256.  Host code only (no device, no handle). */
int zbhip_doc_merge_order(const uint32_t* key_offsets, size_t n, zbhip_doc_entry* entries);

typedef struct zbhip_command {
  uint32_t instance;    /* instance slot; CREATE: the slot to create the instance in */
  uint8_t kind;         /* zbhip_command_kind */
  uint8_t doc_count;    /* entries of the variable document (0 = empty document) */
  uint16_t ref;         /* CREATE: process index; JOB_COMPLETE: job key ordinal in the instance */
  uint32_t doc_begin;   /* first entry in the window's document array */
  uint32_t pad;
} zbhip_command;

/* A cross-partition subscription command (the compact form of the MessageSubscriptionRecord /
 * ProcessMessageSubscriptionRecord that SubscriptionCommandSender.java:54-338 sends with
 * InterPartitionCommandSender; the exchange between partitions moves these, 48 bytes each).
 * Keys are the reference's (relabelled) keys; (instance, element_ord) is the routing handle of the
 * subscribing element instance on its PI partition.  Name ids (message name, bpmnProcessId) and
 * string ids (correlation key) are valid on every partition when deployments and interning are
 * replicated in the same order on all partitions (the host adapter's duty, like deployment
 * distribution). */
typedef struct zbhip_xpart_cmd {
  int64_t element_instance_key;
  int64_t process_instance_key;
  int64_t message_key;       /* -1 unset */
  uint32_t correlation_key;  /* string id (routing: also set where the record value has none) */
  uint32_t instance;         /* PI instance slot on the PI partition */
  uint16_t element_ord;      /* key ordinal of the subscribing element instance in that instance */
  uint16_t message_name;     /* name id */
  uint16_t bpmn_process_id;  /* name id */
  uint8_t kind;              /* ZBHIP_CMD_MSG_SUB_CREATE .. ZBHIP_CMD_MSG_SUB_CORRELATE,
                                ZBHIP_CMD_MSG_SUB_DELETE, ZBHIP_CMD_PMS_DELETE */
  uint8_t interrupting;
  int16_t source_partition;
  int16_t target_partition;
  uint32_t pad;
} zbhip_xpart_cmd;

/* Submits a window of commands in log order.  Host buffers are copied.  Commands of one subject run
 * in log order (the window is split into launches); a CREATE into an instance slot that an earlier
 * command of the same window addresses is refused (ZBHIP_EINVAL): a slot is reused only after the
 * window that ended its instance was drained. */
int zbhip_submit(zbhip_handle* h, const zbhip_command* cmds, size_t n, const zbhip_doc_entry* docs,
                 size_t n_docs);
/* Same, with the window's received cross-partition commands (referenced by doc_begin). */
int zbhip_submit_ex(zbhip_handle* h, const zbhip_command* cmds, size_t n, const zbhip_doc_entry* docs,
                    size_t n_docs, const zbhip_xpart_cmd* xparts, size_t n_xparts);
/* Same, from device-resident arrays already in HBM (no copy; they must stay valid until the next
 * submit, or until zbhip_run returns for a run that reads results back).  The window's subjects are
 * checked on the device (k_subject_check): a window that addresses a subject (instance slot /
 * correlation slot) more than once is copied to the host and planned into rounds like a host window;
 * a subject out of range refuses the window (ZBHIP_EINVAL).  On a partition without messages the check
 * is speculative -- no host wait: a ZBHIP_RUN_NO_RESULTS run launches k_step guarded by the device's
 * verdict, and the next submit (or advance / stats call) reads it and replays a refused window before
 * anything else, reporting ZBHIP_EINVAL there for a subject out of range.  Handles opened with
 * ZBHIP_OPEN_TRUSTED_DEVICE_WINDOWS skip the check: the caller then guarantees one command per
 * subject (the benchmark's windows, by construction). */
int zbhip_submit_device(zbhip_handle* h, const zbhip_command* dev_cmds, size_t n,
                        const zbhip_doc_entry* dev_docs, size_t n_docs);
int zbhip_submit_device_ex(zbhip_handle* h, const zbhip_command* dev_cmds, size_t n,
                           const zbhip_doc_entry* dev_docs, size_t n_docs,
                           const zbhip_xpart_cmd* dev_xparts, size_t n_xparts);

/* Value dictionary (correlation keys and other string variable values): returns the id (>= 0) of
 * the string, interning it if new, or an error.  The device holds each string's Java hashCode
 * (SubscriptionUtil.getSubscriptionHashCode, signed bytes) for subscription routing. */
int64_t zbhip_intern_string(zbhip_handle* h, const char* bytes, size_t len);
/* The list dictionary (ZBHIP_DOC_LIST values: arrays of scalar items -- a multi-instance inputCollection
 * variable, an outputCollection): the id of the list `items` (type, value; name unused; STR values are
 * value-dictionary ids), deduplicated; ZBHIP_EUNSUPP for nested lists.  zbhip_list_items: its items
 * (*n_out = the count, at most cap written). */
int64_t zbhip_intern_list(zbhip_handle* h, const zbhip_doc_entry* items, size_t n);
int zbhip_list_items(zbhip_handle* h, int64_t id, zbhip_doc_entry* out, size_t cap, size_t* n_out);
/* Bulk form: n strings, string i = bytes[offsets[i] .. offsets[i+1]); ids_out may be NULL. */
int zbhip_intern_strings(zbhip_handle* h, const char* bytes, const uint64_t* offsets, size_t n, uint32_t* ids_out);
const char* zbhip_string_value(zbhip_handle* h, uint32_t id, size_t* len);
/* SubscriptionUtil.getSubscriptionPartitionId (protocol-impl/.../SubscriptionUtil.java:22-44). */
int32_t zbhip_subscription_partition(const char* bytes, size_t len, int32_t partition_count);

#define ZBHIP_RUN_NO_RESULTS 1u  /* benchmarking: no D2H copy, no host wait, no key relabelling */
#define ZBHIP_RUN_TIMED 2u       /* record HIP events around the lifecycle kernel launches */
#define ZBHIP_RUN_ACCUMULATE 4u  /* keep accumulating statistics/timings of the previous runs */
#define ZBHIP_RUN_DEVICE_RECORDS 8u /* results mode, but the records stay in HBM until a drain needs them
                                       (zbhip_serialize_log_device reads them there) */
/* Processes the submitted window to quiescence.  Returns #commands processed or <0. */
int zbhip_run(zbhip_handle* h, uint32_t flags);
/* ActorClock.currentTimeMillis() for the next runs: timer catch events get dueDate = now + their
 * duration (CatchEventBehavior.subscribeToTimerEvent, CatchEventBehavior.java:303-330). */
int zbhip_set_clock(zbhip_handle* h, int64_t now_ms);

/* ---- results ------------------------------------------------------------- */
/* Drained record (one per follow-up record of a batch), ordered by (source, ordinal). */
typedef struct zbhip_record {
  int64_t key;                  /* relabelled to the reference key */
  int64_t scope_key;            /* PI: flowScopeKey; JOB: elementInstanceKey; VARIABLE/PROCESS_EVENT:
                                   scopeKey; PI_CREATION: processInstanceKey;
                                   PROCESS_INSTANCE_BATCH: batchElementInstanceKey */
  int64_t process_instance_key;
  int64_t source_index;         /* index of the batch's initial command in submission order */
  int32_t process_idx;
  int32_t element_idx;          /* element/flow index; VARIABLE: variable-name id; -1 none */
  uint8_t record_type;
  uint8_t value_type;
  uint8_t intent;
  uint8_t rejection_type;       /* ZBHIP_REJ_NONE unless record_type == REJECTION */
  uint16_t ordinal;             /* position within the batch */
  uint8_t reason;               /* rejection reason kind (zbhip_reason), 0 = none */
  uint8_t reason_arg;           /* e.g. the offending element-instance state */
  int64_t aux;                  /* VARIABLE: document entry index, or ZBHIP_AUX_INLINE (the value in
                                   message_key, its zbhip_doc_type in partition: multi-instance
                                   loopCounter / input element); JOB:COMPLETED: source doc; INCIDENT: the
                                   sequence flow whose condition was not a boolean (-1: none chosen); else -1 */
  /* message value fields (MESSAGE / MESSAGE_SUBSCRIPTION / PROCESS_MESSAGE_SUBSCRIPTION); a JOB
     record of an ACTIVATED job (JOB:COMPLETED / CANCELED write the stored job): its deadline and worker */
  int64_t message_key;          /* messageKey / JOB: deadline; -1 unset */
  uint32_t correlation_key;     /* string id (JOB: the worker), ZBHIP_NO_STRING = empty */
  uint16_t message_name;        /* name id, 0xFFFF = empty */
  uint16_t bpmn_process_id;     /* name id, 0xFFFF = empty */
  int32_t partition;            /* PMS: subscriptionPartitionId; TIMER events: repetitions (-1 infinite);
                                   INCIDENT: the ErrorType ordinal (reason_arg: the ZBHIP_FEEL_* result);
                                   PROCESS_INSTANCE_BATCH: index (the children still to activate);
                                   VARIABLE with aux == ZBHIP_AUX_INLINE: the value's zbhip_doc_type; else 0 */
  uint8_t interrupting;
  uint8_t unprocessed;          /* a follow-up COMMAND written to the log unprocessed (past
                                   maxCommandsInBatch, ProcessingStateMachine.java:388-417): it
                                   starts a batch of its own later (no skipProcessing flag) */
  uint8_t pad[2];
} zbhip_record;
#define ZBHIP_NO_STRING 0xFFFFFFFFu
#define ZBHIP_AUX_INLINE (-2)

int zbhip_drain(zbhip_handle* h, zbhip_record* out, size_t cap, size_t* n_out);
/* The errorMessage of a drained INCIDENT record (BpmnIncidentBehavior.createIncident's Failure):
 * CONDITION_ERROR "Expected at least one condition to evaluate to true, or to have a default flow"
 * (ExclusiveGatewayProcessor.java:121-125), EXTRACT_VALUE_ERROR "Expected result of the expression
 * '<text>' to be 'BOOLEAN', but was '<NULL|NUMBER|STRING>'." (ExpressionProcessor.java:356-368).
 * Writes at most cap bytes (no NUL) and returns the full length, or < 0. */
int64_t zbhip_incident_message(zbhip_handle* h, const zbhip_record* r, char* out, size_t cap);
/* The records of window command i only: what a host adapter emits when the platform reaches
 * command i (message partitions too: a message record is one zbhip_record, as in zbhip_drain).  Keys of the commands after a fallback
 * command are fixed once the CPU engine's keys for it are declared (zbhip_set_external_keys), so a
 * command after an undeclared fallback returns ZBHIP_ESTATE; zbhip_drain, by contrast, fixes the
 * whole window (undeclared fallbacks generated no keys).  cap too small: ZBHIP_ENOMEM with *n_out =
 * the records needed.  With ZBHIP_OPEN_DEFER_CONTINUATIONS a record written unprocessed carries its
 * continuation id in aux. */
int zbhip_drain_command(zbhip_handle* h, size_t i, zbhip_record* out, size_t cap, size_t* n_out);
/* Number of records the last run produced (before draining). */
int64_t zbhip_pending_records(zbhip_handle* h);

typedef struct zbhip_stats {
  uint64_t commands;            /* commands processed by the last run */
  uint64_t records;             /* records emitted */
  uint64_t transitions;         /* PI events with element-lifecycle/SFT intents */
  uint64_t completed_instances; /* PROCESS ELEMENT_COMPLETED */
  uint64_t keys;                /* keys generated */
  uint64_t fallback;            /* batches flagged for the fallback path */
  double step_ms;               /* device time of the lifecycle kernel launches (ZBHIP_RUN_TIMED runs) */
  double compact_ms;            /* 0: record compaction is fused into the lifecycle kernel */
  uint32_t rounds;              /* per-instance serialisation rounds of the window */
  uint32_t launches;
  uint64_t template_batches;    /* CREATE batches copied from a recorded template (kernels.hip tpl_create) */
} zbhip_stats;
int zbhip_get_stats(zbhip_handle* h, zbhip_stats* out);

/* Exports the partition state as canonical text rows, one per zb-db column-family
 * entry ("CF|key parts|value fields"), keys relabelled; the sink is called per row. */
typedef void (*zbhip_state_sink)(void* ctx, const char* row);
int zbhip_export_state(zbhip_handle* h, zbhip_state_sink sink, void* ctx);

/* Cross-partition commands the last run sent (post-commit side effects of its batches, in log
 * order, keys relabelled); the host routes them to their target partitions (drain mode). */
int zbhip_outbox(zbhip_handle* h, zbhip_xpart_cmd* out, size_t cap, size_t* n_out);
/* The cross-partition commands window command i sent (its batch's post-commit side effects,
 * SubscriptionCommandSender.java:320-338, in batch order; keys relabelled): what a host adapter hands
 * to InterPartitionCommandSender.sendCommand (stream/api/InterPartitionCommandSender.java) once the
 * platform committed command i's batch.  cap too small: ZBHIP_ENOMEM with *n_out = the entries. */
int zbhip_outbox_command(zbhip_handle* h, size_t i, zbhip_xpart_cmd* out, size_t cap, size_t* n_out);
/* Device form: after zbhip_run (any mode) the outbox bucketed by target partition, stable in log
 * order, with device-computed keys; counts[t] = entries for partition t + 1 (partition_count
 * entries).  The pointer stays valid until the next run.  This is what the RCCL all-to-all sends.
 * The outbox is handed out once: later calls before the next run report zero counts. */
int zbhip_outbox_device(zbhip_handle* h, const zbhip_xpart_cmd** dev_out, uint32_t* counts);

/* Same without a host wait: the per-target counts (uint32[partition_count]) are copied to dev_counts
 * (device memory) asynchronously on the handle's stream -- what a device-resident all-to-all
 * exchange feeds to its count collective, so an exchange round needs a single host sync. */
int zbhip_outbox_device_async(zbhip_handle* h, const zbhip_xpart_cmd** dev_out, void* dev_counts);

/* The hipStream_t the handle launches on (the configured stream, or the handle's own): callers that
 * order their own device work against the handle's (an exchange's collectives) use this stream. */
void* zbhip_stream(zbhip_handle* h);

/* Copies bucketed outbox entries [first, first + count) (zbhip_outbox_device order) to dev_dst,
 * asynchronously on the handle's stream. */
int zbhip_outbox_copy(zbhip_handle* h, void* dev_dst, size_t first, size_t count);
/* The exchange of several partitions hosted by one process on one GPU, in one launch: target t's
 * inbox dst[t] receives, for every source s in partition order, the count[s][t] entries of s's
 * bucketed outbox (zbhip_outbox_device_async's pointer src[s]) bound for t -- the arrival order of
 * DeviceExchange.  dev_counts: [P][P] uint32 in device memory (the sources' count rows); max_count
 * bounds its entries (grid size); P <= 16; launched on `stream` (a hipStream_t, NULL = default). */
int zbhip_exchange_gather(const zbhip_xpart_cmd* const* src, uint32_t P, const uint32_t* dev_counts,
                          zbhip_xpart_cmd* const* dst, uint32_t max_count, void* stream);
/* Receiving side of the exchange: submits the n received commands at dev_xparts (device memory,
 * arrival order) as the next window, building its commands on the device (subject = the PI
 * instance slot for PROCESS_MESSAGE_SUBSCRIPTION commands, the correlation slot otherwise).
 * dev_xparts must stay valid until zbhip_run returns. */
int zbhip_submit_xparts_device(zbhip_handle* h, const zbhip_xpart_cmd* dev_xparts, size_t n);
/* SubscriptionUtil.getSubscriptionPartitionId of n interned strings (out[i] in 1..partition_count). */
int zbhip_string_partitions(zbhip_handle* h, const uint32_t* ids, size_t n, int32_t partition_count, int32_t* out);

/* Instances whose last batch needs the fallback path (incident, FEEL outside the
 * subset, batch-limit overflow, capacity).  Their state was left untouched. */
int zbhip_fallback(zbhip_handle* h, uint32_t* instances, size_t cap, size_t* n_out);

/* ZBHIP_OPEN_DEFER_CONTINUATIONS: the continuation ids the last run handed out, [first, first + n),
 * one per drained record with `unprocessed` set, in drain order. */
int zbhip_continuations(zbhip_handle* h, uint64_t* first_id, uint64_t* n);
/* Continuations of the instance in slot `instance` still waiting to be read back: its slot is not
 * free for a CREATE until they ran (or the instance was evicted, which drops them). */
int zbhip_pending_continuations(zbhip_handle* h, uint32_t instance);

/* DbKeyGenerator between windows (stream-platform/.../state/DbKeyGenerator.java:39-61).  The
 * partition has one key generator: the host keeps the reference's (the CPU engine's, in RocksDB)
 * level with the device's.  zbhip_current_key: the last key generated so far (the last window's keys
 * and the CPU engine's declared ones); zbhip_set_key_if_higher: keys the CPU engine generated
 * between windows (KeyGeneratorControls.setKeyIfHigher), the next window's follow them. */
int zbhip_current_key(zbhip_handle* h, int64_t* key);
int zbhip_set_key_if_higher(zbhip_handle* h, int64_t key);

/* Status of command i of the last run: 0 = processed, 1 = needs the fallback path; *reason is
 * the device fallback code (FB_* in zeebe_amd/csrc/zb_internal.h), 0 when processed. */
int zbhip_command_status(zbhip_handle* h, size_t i, uint32_t* status, uint32_t* reason);

/* Maps a drained (relabelled) key back to (instance, key ordinal) for building
 * follow-up commands (e.g. JOB:COMPLETE).  Returns ZBHIP_EINVAL if unknown or if the instance that
 * generated it has ended (its slot may hold a new instance): the adapter hands such a command to the
 * CPU engine, which rejects it (NOT_FOUND) as the reference does. */
int zbhip_resolve_key(zbhip_handle* h, int64_t key, uint32_t* instance, uint16_t* ordinal);

/* Rejection reasons (text formats in zbhip_rejection_reason). */
enum zbhip_reason {
  ZBHIP_REASON_NONE = 0,
  ZBHIP_REASON_PGW_NOT_ALL_TAKEN = 1, /* ProcessInstanceStateTransitionGuard.java:169-186 */
  ZBHIP_REASON_FS_NOT_FOUND = 2,      /* :88-100 */
  ZBHIP_REASON_FS_STATE = 3,          /* :116-128 */
  ZBHIP_REASON_EI_NOT_FOUND = 4,      /* :74-86 */
  ZBHIP_REASON_EI_STATE = 5,          /* :102-114 */
  ZBHIP_REASON_JOB_NOT_FOUND = 6,     /* JobCommandPreconditionChecker.java */
  ZBHIP_REASON_MS_ALREADY_OPEN = 7,   /* MessageSubscriptionCreateProcessor SUBSCRIPTION_ALREADY_OPENED_MESSAGE */
  ZBHIP_REASON_PMS_CREATE_NOT_FOUND = 8, /* ProcessMessageSubscriptionCreateProcessor NO_SUBSCRIPTION_FOUND */
  ZBHIP_REASON_PMS_CREATE_NOT_OPENING = 9, /* ... NOT_OPENING_MSG ("opened"/"closing") */
  ZBHIP_REASON_PMS_CORR_NOT_FOUND = 10, /* ProcessMessageSubscriptionCorrelateProcessor NO_SUBSCRIPTION_FOUND */
  ZBHIP_REASON_PMS_CORR_NO_EVENT = 11,  /* ... NO_EVENT_OCCURRED_MESSAGE */
  ZBHIP_REASON_MS_CORR_NOT_FOUND = 12,  /* MessageSubscriptionCorrelateProcessor NO_SUBSCRIPTION_FOUND */
  ZBHIP_REASON_TIMER_NOT_FOUND = 13,    /* TriggerTimerProcessor NO_TIMER_FOUND_MESSAGE */
  ZBHIP_REASON_TIMER_NOT_ACTIVE = 14,   /* TriggerTimerProcessor NO_ACTIVE_TIMER_MESSAGE */
  ZBHIP_REASON_JOB_TIME_OUT = 15,       /* JobTimeOutProcessor NOT_ACTIVATED_JOB_MESSAGE; reason_arg 0 "no such job
                                           was found", 1 "it must be activated first", 2 "it has not timed out" */
  ZBHIP_REASON_JOB_STATE = 16           /* JobCommandPreconditionChecker (:33-49) of the record's intent: reason_arg =
                                           the JobState.State (2 FAILED: "it is in state 'FAILED'", 3 NOT_FOUND) */
};
/* Rejection reason text exactly as the reference writes it. */
int zbhip_rejection_reason(zbhip_handle* h, const zbhip_record* rec, char* buf, size_t cap);

/* ---- log serialisation --------------------------------------------------
 * Drained records -> the bytes the reference's log stream holds for them: per source command one
 * sequenced batch (SequencedBatchSerializer.java:33-67) of 8-aligned entries, each = dispatcher
 * frame (DataFrameDescriptor.java, 12 bytes) + LogEntryDescriptor header (40 bytes: flags with
 * skipProcessing for processed follow-up commands, position, sourcePosition, key, timestamp,
 * metadata length) + SBE RecordMetadata (protocol.xml:137-152, schema version 4) + msgpack record
 * value (ObjectValue.java:78-84; ProcessInstanceRecord, JobRecord, VariableRecord,
 * ProcessEventRecord, ProcessInstanceCreationRecord, MessageRecord, MessageSubscriptionRecord,
 * ProcessMessageSubscriptionRecord).  Host code (no device work).
 * A serializer holds the deployment's constant msgpack runs and the name / value dictionaries; a
 * handle owns one kept in step with zbhip_deploy / zbhip_intern / zbhip_intern_string
 * (zbhip_handle_serializer), a standalone one is built with the same calls in the same order. */
typedef struct zbhip_serializer zbhip_serializer;
int zbhip_serializer_new(zbhip_serializer** out);
void zbhip_serializer_free(zbhip_serializer* s);
int zbhip_serializer_deploy(zbhip_serializer* s, const zbhip_process_csr* csr, uint32_t* process_idx_out);
int zbhip_serializer_intern(zbhip_serializer* s, const char* name);
int64_t zbhip_serializer_intern_string(zbhip_serializer* s, const char* bytes, size_t len);
/* the list dictionary (ZBHIP_DOC_LIST values), in the handle's id order: items as zbhip_doc_entry rows
 * (type, value; name unused) */
int64_t zbhip_serializer_intern_list(zbhip_serializer* s, const zbhip_doc_entry* items, size_t n);
/* RecordMetadata.brokerVersion written into every entry (default 8.4.0, the reference build). */
int zbhip_serializer_set_broker_version(zbhip_serializer* s, int32_t major, int32_t minor, int32_t patch);
int zbhip_serializer_rejection_reason(zbhip_serializer* s, const zbhip_record* rec, char* buf, size_t cap);
/* zbhip_incident_message on a serializer's deployments. */
int64_t zbhip_serializer_incident_message(zbhip_serializer* s, const zbhip_record* rec, char* buf, size_t cap);
zbhip_serializer* zbhip_handle_serializer(zbhip_handle* h);

/* The window the records were drained from, and the log positions of its batches. */
/* The TimerRecord of a TIMER:TRIGGER command as DueDateTimerChecker wrote it
 * (engine/.../processing/timer/DueDateTimerChecker.java:118-125: the stored timer's keys, element,
 * repetitions); a rejection of the command carries it (TypedRejectionWriter.appendRejection). */
typedef struct zbhip_timer_value {
  int64_t element_instance_key;
  int64_t process_instance_key;
  int64_t process_definition_key;
  int32_t repetitions;
  int32_t process_idx;           /* targetElementId = element element_idx of this process; -1 = "" */
  int32_t element_idx;
  int32_t pad;
} zbhip_timer_value;

typedef struct zbhip_log_window {
  const zbhip_command* cmds;       /* the submitted window (record.source_index - source_base) */
  size_t n_cmds;
  int64_t source_base;             /* source_index of cmds[0] */
  const zbhip_doc_entry* docs;     /* its document entries (record.aux - doc_base for VARIABLE) */
  size_t n_docs;
  int64_t doc_base;
  const int64_t* source_positions; /* log position of each command of the window (sourcePosition) */
  int64_t first_position;          /* position of the first serialised record (the sequencer's next) */
  int64_t timestamp;               /* the batches' timestamp (ms) */
  const int64_t* source_timestamps;/* timestamp of each window command (MESSAGE deadline =
                                      PUBLISH timestamp + timeToLive); NULL = timestamp */
  const zbhip_timer_value* timer_values; /* per window command: a TIMER:TRIGGER's TimerRecord, written
                                      for its rejection; NULL = the window's key and dueDate only (the
                                      device form then leaves such windows to the host serialiser) */
} zbhip_log_window;

/* Serialises n drained records (in drain order) into out.  *used = bytes needed; ZBHIP_ENOMEM if
 * cap is short (out == NULL: size query). */
int zbhip_serialize_log(zbhip_serializer* s, const zbhip_record* recs, size_t n, const zbhip_log_window* w,
                        uint8_t* out, size_t cap, size_t* used);

/* Device form (configs 1-4): after zbhip_run with results, every record of the window serialised
 * into device memory (owned by the handle, valid until the next call) -- the same bytes as
 * zbhip_drain + zbhip_serialize_log(zbhip_handle_serializer(h), ...) with this window description
 * (w->cmds / w->docs / bases are taken from the handle; w->source_positions, first_position,
 * timestamp are used).  Keys are relabelled on the device: ordinals of the batch from its key base,
 * older ones from a per-instance ring of the last 16 ordinals in HBM, which holds every key only if
 * every window of the handle comes through here.  ZBHIP_EUNSUPP (use the host serialiser for this
 * window and the later ones): message partitions, continuation batches, imported state, string
 * variables, a key older than the ring, or a window that skipped this call.  The bytes are written
 * asynchronously in the order of the handle's stream (zbhip_stream): zbhip_log_device_copy and the
 * handle's next run wait for them; a reader on another stream waits on that stream first. */
int zbhip_serialize_log_device(zbhip_handle* h, const zbhip_log_window* w, const void** dev_bytes, size_t* used);
/* Copies n bytes of the last zbhip_serialize_log_device output into host memory. */
int zbhip_log_device_copy(zbhip_handle* h, void* dst, size_t n);
/* The log bytes into host memory without a wait (LogStorage.append's input on the host): the n bytes of the
 * last zbhip_serialize_log_device output are copied on a copy stream of the handle, after the write, into a
 * pinned buffer the handle owns; *host_bytes is where they land.  From the first call on the handle keeps two
 * device output buffers and two pinned ones used in turn, so window k's bytes cross PCIe while window k+1 is
 * submitted, run and serialised (the write of window k+2 waits for copy k).  The bytes are complete once
 * zbhip_log_copy_wait(h, *host_bytes) returns and stay valid until the second next zbhip_log_copy_async
 * (NULL waits for every pending copy). */
int zbhip_log_copy_async(zbhip_handle* h, size_t n, const void** host_bytes);
int zbhip_log_copy_wait(zbhip_handle* h, const void* host_bytes);

/* ---- zb-db byte encoding of the state ---------------------------------------
 * The partition state as RocksDB entries: key = 8-byte big-endian ZbColumnFamilies ordinal +
 * DbLong / DbString / DbInt parts, value = DbNil / DbLong / DbInt or the msgpack of the state
 * object (ElementInstance, VariableInstance, EventScopeInstance, JobRecordValue, JobStateValue,
 * NextValue, MessageSubscription, ProcessMessageSubscription) -- the 15 column families of the path. */
typedef void (*zbhip_db_sink)(void* ctx, uint32_t column_family, const uint8_t* key, size_t key_len,
                              const uint8_t* value, size_t value_len);
int zbhip_export_state_db(zbhip_handle* h, zbhip_db_sink sink, void* ctx);
/* One canonical row of zbhip_export_state -> its entry; 1 = emitted, 0 = column family not encoded. */
int zbhip_serializer_encode_state_row(zbhip_serializer* s, const char* row, zbhip_db_sink sink, void* ctx);

/* ---- job activation ----------------------------------------------------------
 * JOB_BATCH:ACTIVATE (JobBatchActivateProcessor.java:60-143, JobBatchCollector.java:67-123,
 * JobBatchActivatedApplier.java:27-37, DbJobState.activate :118-133): the activatable jobs of a type
 * in JOB_ACTIVATABLE order (job key) up to maxJobsToActivate, each with deadline = the command's
 * timestamp + timeout, the worker, and the variables visible from its element instance
 * (JobVariablesCollector / DbVariableState.getVariablesAsDocument: the element's scope, then the
 * process instance's, names in DbString order -- length, then bytes -- each name once, filtered by
 * the requested names if any); the jobs become ACTIVATED (JOB_STATES, JOB_DEADLINES, out of
 * JOB_ACTIVATABLE).  The batch key is the partition's next key.  A command is processed between
 * windows, in log order.  The size-based truncation of the reference (4 MB records) is not modelled:
 * at most `cap` jobs are returned. */
typedef struct zbhip_job_activation {
  const char* type;            /* job type (UTF-8) */
  size_t type_len;
  const char* worker;
  size_t worker_len;
  int64_t timeout;             /* ms */
  int32_t max_jobs;            /* maxJobsToActivate */
  int32_t pad;
  int64_t timestamp;           /* the command's timestamp (ms) */
  const uint32_t* variables;   /* requested variable name ids (zbhip_intern); none = every variable */
  size_t n_variables;
} zbhip_job_activation;

typedef struct zbhip_activated_job {
  int64_t key;                   /* job key */
  int64_t element_instance_key;
  int64_t process_instance_key;
  int64_t deadline;
  uint32_t instance;             /* instance slot */
  int32_t process_idx;
  int32_t element_idx;
  uint16_t retries;
  uint16_t n_variables;
  zbhip_doc_entry variables[6];  /* the job's variables document, in document order */
} zbhip_activated_job;

typedef struct zbhip_job_batch {
  int64_t key;                   /* JOB_BATCH:ACTIVATED key; -1 when rejected */
  uint32_t n_jobs;
  uint8_t rejection_type;        /* ZBHIP_REJ_INVALID_ARGUMENT or ZBHIP_REJ_NONE */
  uint8_t reason;                /* 1 max jobs, 2 timeout, 3 type (JobBatchActivateProcessor.rejectCommand) */
  uint8_t truncated;
  uint8_t pad;
} zbhip_job_batch;

int zbhip_activate_jobs(zbhip_handle* h, const zbhip_job_activation* cmd, zbhip_activated_job* jobs, size_t cap,
                        zbhip_job_batch* result);
/* The device's JOB_ACTIVATABLE keys of a job type in key order (DbJobState.forEachActivatableJobs,
 * state/instance/DbJobState.java:231-252, over the device's jobs): at most cap into keys, *n_out the
 * count.  A host whose engine holds jobs of the same type (handed-off instances) merges both lists and
 * activates each side's share -- the engine's first (its nextKey is the batch key), then
 * zbhip_activate_jobs with the device's, which takes the same key. */
int zbhip_activatable_jobs(zbhip_handle* h, const char* type, size_t type_len, int64_t* keys, size_t cap, size_t* n_out);
/* The push side effect of a job stream (BpmnJobActivationBehavior.java:83-97: JobVariablesCollector over
 * the stream's fetchVariables, then JobStream.push of the ActivatedJob): for each of the n job keys (the
 * aux of the JOB_BATCH:ACTIVATED records a run or zbhip_time_out_job / zbhip_fail_job wrote), its
 * activation and variables document (`names`: the fetchVariables name ids, none = every variable) into
 * out[i]; key -1 for a key that is no live device job.  Reads device state only. */
int zbhip_job_variables(zbhip_handle* h, const int64_t* job_keys, size_t n, const uint32_t* names, size_t n_names,
                        zbhip_activated_job* out);
/* The rejection reason of a refused JOB_BATCH:ACTIVATE, exactly as JobBatchActivateProcessor writes it. */
int zbhip_job_batch_rejection_reason(const zbhip_job_activation* cmd, const zbhip_job_batch* result, char* buf, size_t cap);

/* ---- the engine's scheduled tasks over device-held state ---------------------------------------
 * The reference's checkers scan RocksDB, which does not hold what the device holds; a host adapter's
 * checkers read these instead and write the same commands.  Call them between
 * batches once the current window's commands were all emitted (zbhip_drain_command): the device state
 * is then exactly the log's.  Records come back as zbhip_record rows, so the adapter builds the
 * command values with the same code as drained records. */
/* DueDateTimerChecker.TriggerTimersSideEffect (processing/timer/DueDateTimerChecker.java:86-129) ->
 * DbTimerInstanceState.processTimersWithDueDateBefore (state/instance/DbTimerInstanceState.java:87-116):
 * the TIMER:TRIGGER commands of the device timers with dueDate <= now, in TIMER_DUE_DATES order
 * (dueDate, elementInstanceKey, timer key); at most cap, *next_due = the first dueDate not returned
 * (-1: none) -- what DueDateChecker reschedules with.  A device scan (k_due_timers, 16 B per instance).
 * Truncated (n == cap and *next_due <= now: due rows were left out), a merge with the engine's
 * TIMER_DUE_DATES visits the engine's timers only up to the last row returned and stops there
 * (processTimersWithDueDateBefore may stop at any timer; the checker runs again at the returned date). */
int zbhip_due_timers(zbhip_handle* h, int64_t now, zbhip_record* out, size_t cap, size_t* n_out, int64_t* next_due);
/* JobTimeoutTrigger.DeactivateTimeOutJobs (processing/job/JobTimeoutTrigger.java:74-87) ->
 * DbJobState.forEachTimedOutEntry (state/instance/DbJobState.java:286-298): the JOB:TIME_OUT commands
 * (key = the job, value = the stored job) of ACTIVATED device jobs with deadline < now, in JOB_DEADLINES
 * order (deadline, key); at most cap, *next_deadline = the deadline of the first timed-out job not returned
 * (-1: none were left out; NULL allowed).  A merge with the engine's JOB_DEADLINES then visits the
 * engine's entries only up to the last row returned (the rest come with the trigger's next run). */
int zbhip_timed_out_jobs(zbhip_handle* h, int64_t now, zbhip_record* out, size_t cap, size_t* n_out,
                         int64_t* next_deadline);
/* JOB:TIME_OUT of a device job (JobTimeOutProcessor.processRecord, processing/job/JobTimeOutProcessor
 * .java:46-73; `now` = ActorClock.currentTimeMillis()): out[0] = JOB:TIMED_OUT with the stored job
 * (JobTimedOutApplier -> DbJobState.timeout: ACTIVATABLE again, deadline and worker kept) and, with a job
 * stream of its type, out[1] = its push (publishWork); or the NOT_FOUND rejection (reason
 * ZBHIP_REASON_JOB_TIME_OUT; the adapter writes the command's value).  cap >= 2. */
int zbhip_time_out_job(zbhip_handle* h, int64_t job_key, int64_t now, zbhip_record* out, size_t cap, size_t* n_out);
/* A job stream for a job type (JobStreamer.streamFor: a gateway's StreamActivatedJobs with its worker and
 * timeout; on = 0 removes it).  From the next run on, a job a device batch creates of that type is pushed
 * as BpmnJobActivationBehavior.publishWork (processing/bpmn/behavior/BpmnJobActivationBehavior.java:61-100)
 * does: JOB_BATCH:ACTIVATED (key = the next key) right after JOB:CREATED, the job ACTIVATED with deadline =
 * the run's clock + timeout and the worker (drained record: value_type ZBHIP_VT_JOB_BATCH, aux = the job
 * key, the job's fields as a JOB record's).  zbhip_time_out_job and zbhip_fail_job (retries left) push the
 * same way.  Tasks with a stream run on the general path (no straight-line segment). */
int zbhip_set_job_stream(zbhip_handle* h, const char* type, size_t type_len, const char* worker, size_t worker_len,
                         int64_t timeout, int on);
/* JOB:FAIL of a device job (JobFailProcessor.processRecord / failJob, processing/job/JobFailProcessor.java
 * :79-162; JobFailedApplier -> DbJobState.fail :191-203).  out[0] = JOB:FAILED (the stored job with the
 * command's retries and errorMessage -- StringUtil.limitString at 10 000 -- JOB records: reason_arg bit 0 =
 * partition holds the retries and message_name | bpmn_process_id << 16 the errorMessage's string id) or
 * the rejection (NOT_FOUND / INVALID_STATE, reason ZBHIP_REASON_JOB_STATE); retries <= 0: out[1] =
 * INCIDENT:CREATED (ErrorType JOB_NO_RETRIES in partition, aux = the job key, correlation_key = the
 * errorMessage's id: the job's, or "No more retries left."; key = the next key) and the job is FAILED.
 * ACTIVATABLE again with retries left; a later activation keeps the retries.  Returns ZBHIP_EUNSUPP for
 * commands outside the subset (variables, a retry back-off): the adapter hands the instance to the
 * engine.  cap >= 2. */
typedef struct zbhip_job_fail {
  int64_t job_key;
  int64_t retry_backoff;
  int64_t timestamp;      /* the command's (ActorClock): a push's deadline */
  const char* error_message;
  size_t error_message_len;
  int32_t retries;
  uint32_t n_variables;   /* entries of the command's variable document */
} zbhip_job_fail;
int zbhip_fail_job(zbhip_handle* h, const zbhip_job_fail* cmd, zbhip_record* out, size_t cap, size_t* n_out);
/* The JobState.State of a device job with stored fields: 0 ACTIVATABLE, 1 ACTIVATED, 2 FAILED, 3 gone; -1 none
 * stored (ACTIVATABLE if the key is a live job's).  The adapter rejects JOB:COMPLETE of a FAILED job itself. */
int zbhip_job_state(zbhip_handle* h, int64_t job_key);

/* ---- fallback hand-off (Engine.java:134 onProcessingError, ProcessingStateMachine.java:276-310) --
 * A command the device did not process (zbhip_command_status != 0) goes to the CPU engine, in log
 * order.  Every later command of the same subject in the window falls back too (FB_FENCED), so the
 * CPU engine sees the subject's commands in log order against the state they were left in.  For
 * each fallback command the adapter
 *   1. moves the instance to the CPU engine once: zbhip_export_instances_db (its zb-db entries, to
 *      be written into RocksDB) + zbhip_evict_instances (the slot is freed, its keys stop resolving);
 *   2. sets DbKeyGenerator to zbhip_key_before(h, i) and runs engine.process(command);
 *   3. declares the keys that generated: zbhip_set_external_keys(h, i, n).
 * Keys of the window's later device-processed commands follow those (relabelled at the first
 * drain / export / resolve, which fixes the window's keys).  Config 5 windows: declared keys must
 * be 0 (the device already fixed their keys for the exchange). */
int zbhip_export_instances(zbhip_handle* h, const uint32_t* instances, size_t n, zbhip_state_sink sink, void* ctx);
int zbhip_export_instances_db(zbhip_handle* h, const uint32_t* instances, size_t n, zbhip_db_sink sink, void* ctx);
int zbhip_evict_instances(zbhip_handle* h, const uint32_t* instances, size_t n);
int zbhip_key_before(zbhip_handle* h, size_t i, int64_t* key);
int zbhip_set_external_keys(zbhip_handle* h, size_t i, uint32_t nkeys);

/* ---- one owner of a correlation key's message state (config 5, the message partition) ----------
 * The reference correlates a publish to every open subscription of [name, correlationKey] and buffers a
 * message with a time-to-live for subscriptions opened later (MessagePublishProcessor.java:83-124,
 * MessageSubscriptionCreateProcessor.java:83-104 -> MessageCorrelator.correlateNextMessage).  The device
 * keeps subscriptions only; a publish outside its subset (a time-to-live, a message id, variables, a
 * name the device's catch events do not wait for) is the engine's, and so from then on is the whole
 * correlation key: before the engine processes that publish the adapter moves the key's correlation
 * slot to the engine -- zbhip_export_correlation_slots(_db) (its MESSAGE_SUBSCRIPTION_BY_KEY /
 * _BY_NAME_AND_CORRELATION_KEY rows, into RocksDB) + zbhip_evict_correlation_slots (the rows freed) --
 * and routes every later message command of that key to the engine. */
int zbhip_export_correlation_slots(zbhip_handle* h, const uint32_t* slots, size_t n, zbhip_state_sink sink, void* ctx);
int zbhip_export_correlation_slots_db(zbhip_handle* h, const uint32_t* slots, size_t n, zbhip_db_sink sink, void* ctx);
int zbhip_evict_correlation_slots(zbhip_handle* h, const uint32_t* slots, size_t n);

/* ---- zb-db bytes back into HBM (restart / hand-back; the reference's
 * replay-equivalence property, ReplayStateRandomizedPropertyTest.java:74-140) ----------------------
 * One zb-db entry -> its canonical state row (the inverse of zbhip_serializer_encode_state_row);
 * string variable values are interned through `intern` (NULL: refused).  Returns the row's length,
 * 0 for a column family outside the path, or an error. */
typedef int64_t (*zbhip_string_interner)(void* ctx, const char* bytes, size_t len);
int zbhip_serializer_decode_state_entry(zbhip_serializer* s, uint32_t column_family, const uint8_t* key, size_t key_len,
                                        const uint8_t* value, size_t value_len, zbhip_string_interner intern,
                                        void* ictx, char* row, size_t cap);
/* Recovery hand-back (StreamProcessorLifecycleAware.onRecovered): of the entries (the format below) of
 * the engine's state, marks in take[i] those of the process instances the handle can take over --
 * instances of processes deployed on it, minus the process instance keys in `exclude` (instances a
 * command still waiting in the log addresses by its own record).  *n_entries = entries read (take
 * needs that many bytes, else ZBHIP_ENOMEM).  Returns the number of instances selected. */
int zbhip_select_instances_db(zbhip_handle* h, const uint8_t* entries, size_t len, const int64_t* exclude,
                              size_t n_exclude, uint8_t* take, size_t n_take, size_t* n_entries);
/* Loads process instances into free instance slots from their zb-db entries (a flat buffer of
 * entries, each: uint32 column family, uint32 key length, uint32 value length, key bytes, value bytes
 * -- the entries zbhip_export_state_db / zbhip_export_instances_db produce, e.g. a RocksDB
 * snapshot's).  The deployments (same definition keys) must be deployed first.  The instances take
 * the slots first_slot, first_slot + 1, ... in process-instance-key order; every key keeps its value
 * (zbhip_resolve_key resolves their job keys and process-instance keys), and the key counter moves
 * to KEY latestKey if that is larger.  *n_instances = instances loaded.  Column families of the
 * message partition side (MESSAGE_SUBSCRIPTION_*) are refused (ZBHIP_EUNSUPP): their routing handles
 * to the subscribers' instance slots are not in the reference's state. */
int zbhip_import_state_db(zbhip_handle* h, const uint8_t* entries, size_t len, uint32_t first_slot,
                          uint32_t* n_instances);
/* The same from canonical state rows (zbhip_export_state's format), '\n'-separated. */
int zbhip_import_state(zbhip_handle* h, const char* rows, size_t len, uint32_t first_slot, uint32_t* n_instances);

/* Library build information ("gfx950 …"). */
const char* zbhip_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* ZBHIP_H */
