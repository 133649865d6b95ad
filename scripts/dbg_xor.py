import sys; sys.path.insert(0,'.')
from tests.helpers import *
from zeebe_amd.engine import Partition
from zeebe_amd import bpmn
def run(xml, with_doc):
    part = Partition(max_instances=4, max_commands=4)
    proc = part.deploy(xml)
    docs=None
    cmds = create_commands(1, proc)
    if with_doc:
        docs = amount_docs([1500], part.intern("amount")); cmds["doc_count"] = 1
    part.submit(cmds, docs); part.run()
    return part.command_status(0), len(part.drain())
xor1 = bpmn.createExecutableProcess("p").startEvent("s").exclusiveGateway("x").endEvent("e").done()
print("linear+doc", run(bpmn.linear_process(2), True))
print("xor1 nodoc", run(xor1, False))
print("xor1 doc", run(xor1, True))
print("xor nodoc", run(bpmn.xor_process(), False))
print("xor doc", run(bpmn.xor_process(), True))
print("xor2 doc", run(bpmn.createExecutableProcess("p").startEvent("s").exclusiveGateway("x").sequenceFlowId("a").conditionExpression("amount > 1").endEvent("e").done(), True))
