"""Debug helper: the PSM non-interrupting boundary test; on the first device fallback, the falling
command and the message partition's subscription rows (device export)."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import test_gpu_psm_messages as T
from psm import Client, open_jobs
from oracle.oracle import subscription_partition
from zeebe_amd import adapter as A

orig = A.GpuBatchProcessor._fall_back


def fb(self, i, record, out):
    print("FALLBACK partition", self.partition_id, "record", record.value_type, record.intent, record.key, dict(record.value))
    for r in self.part.state():
        if r.startswith("MESSAGE_SUBSCRIPTION_BY_KEY") or r.startswith("PROCESS_SUBSCRIPTION_BY_KEY"):
            print("   ", r)
    print("window cmd", self.window.cmds[i])
    raise SystemExit(1)


A.GpuBatchProcessor._fall_back = fb
ref, gpu = T.Cluster(device=False, xml=T.NON_INT_XML), T.Cluster(device=True, xml=T.NON_INT_XML)
T.phase(ref, gpu, T.create_phase("nonIntBoundaryEventProcess"))
pubs = {p: [] for p in range(1, T.P + 1)}
for k in T.KEYS:
    pubs[subscription_partition(k, T.P)] += [Client.publish_message("message", k) for _ in range(3)]
T.phase(ref, gpu, sorted(pubs.items()))
print("after publish: partition 2 rows")
for r in gpu.state(2):
    if r.startswith("MESSAGE_SUBSCRIPTION_BY_KEY"):
        print("   ", r)
jobs = {p: [Client.complete_job(k) for k in sorted(open_jobs(ref.logs[p]))] for p in range(1, T.P + 1)}
T.phase(ref, gpu, sorted(jobs.items()))
print("ok")
