"""Cross-partition subscription exchange.

The reference sends every cross-partition subscription command as a post-commit side effect
through ``InterPartitionCommandSender`` (broker/.../InterPartitionCommandSenderImpl.java:51-100,
one atomix unicast per command; SubscriptionCommandSender.java:304-338).  Here a partition's
run leaves its sent commands in an outbox (48-byte ``zbhip_xpart_cmd``), bucketed on the device
by target partition and stable in log order; one exchange step per protocol phase moves every
bucket to its partition:

* :func:`route` -- host form (drain mode, tests, the in-process multi-partition driver): the
  outboxes of partitions 1..P are concatenated per target in source-partition order;
* :class:`DeviceExchange` -- one process per GPU: ``all_to_all_single`` of the per-target counts
  (P x int64) followed by an all-to-all-v of the 48-byte commands.  With the ``nccl`` backend
  this is RCCL over xGMI: each GPU pair uses its own link, no ring.

The received commands become the next window of the target partition
(:func:`window_from_xparts`): subject = the PI instance slot for PROCESS_MESSAGE_SUBSCRIPTION
commands and the correlation slot for MESSAGE_SUBSCRIPTION commands.
"""
import numpy as np

from . import abi


def window_from_xparts(xp):
    """Commands (log order = arrival order) referencing the received xpart commands by index."""
    xp = np.ascontiguousarray(xp, dtype=abi.XPART_DTYPE)
    cmds = abi.make_commands(len(xp))
    kind = xp["kind"]
    cmds["kind"] = kind
    cmds["doc_begin"] = np.arange(len(xp), dtype=np.uint32)
    pms = (kind == abi.CMD_PMS_CREATE) | (kind == abi.CMD_PMS_CORRELATE)
    cmds["instance"] = np.where(pms, xp["instance"], xp["correlation_key"])
    return cmds, xp


def route(outboxes, partition_count):
    """outboxes[p-1] = xpart array sent by partition p (in its log order).  Returns, per target
    partition, the received xpart array: sources in partition order, each in its send order."""
    inbox = [[] for _ in range(partition_count)]
    for ob in outboxes:
        ob = np.asarray(ob, dtype=abi.XPART_DTYPE)
        for t in range(1, partition_count + 1):
            sel = ob[ob["target_partition"] == t]
            if len(sel):
                inbox[t - 1].append(sel)
    return [np.concatenate(x) if x else abi.make_xparts(0) for x in inbox]


XPART_BYTES = abi.XPART_DTYPE.itemsize


class LocalExchange:
    """Several partitions hosted by one process on one GPU (all on one stream): every target's
    inbox is the concatenation, in source-partition order, of the sources' device buckets for it,
    assembled with device-to-device copies.  ``step()`` returns the inbox sizes; ``deliver()``
    submits each non-empty inbox as the target's next window."""

    def __init__(self, parts, max_entries, device):
        import torch
        self.parts = parts
        self.inbox = [torch.empty(max_entries * XPART_BYTES, dtype=torch.uint8, device=device) for _ in parts]
        self.sizes = [0] * len(parts)

    def step(self):
        P = len(self.parts)
        buckets = [p.outbox_device()[1] for p in self.parts]
        for t in range(P):
            off = 0
            for s_, counts in enumerate(buckets):
                c = int(counts[t])
                if c:
                    first = int(counts[:t].sum())
                    self.parts[s_].outbox_copy(self.inbox[t].data_ptr() + off * XPART_BYTES, first, c)
                    off += c
            self.sizes[t] = off
        return list(self.sizes)

    def deliver(self, flags=0):
        ran = 0
        for t, part in enumerate(self.parts):
            if self.sizes[t]:
                part.submit_xparts_device(self.inbox[t].data_ptr(), self.sizes[t])
                part.run(flags)
                ran += 1
        return ran


class DeviceExchange:
    """All-to-all of device-resident outboxes between the ranks of a process group (rank r =
    partition r + 1).  ``send`` takes the outbox as a uint8 device tensor already bucketed by
    target (``zbhip_outbox_device``) and the per-target counts; it returns the received bucket
    concatenation (uint8 tensor of 48-byte commands, sources in rank order) and its length."""

    XPART_BYTES = abi.XPART_DTYPE.itemsize

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)

    def exchange_partition(self, part, staging, flags=0):
        """One exchange step for this rank's partition: send its device outbox, receive its inbox
        (into ``staging``, a uint8 device tensor), submit and run it.  Returns (received, total
        received over all ranks); every rank calls it the same number of times."""
        import torch
        ptr, counts = part.outbox_device()
        n = int(counts.sum())
        if n:
            part.outbox_copy(staging.data_ptr(), 0, n)
        inbox, got = self.send(staging, counts)
        total = torch.tensor([got], dtype=torch.int64, device=staging.device)
        self.dist.all_reduce(total, group=self.group)
        if got:
            part.submit_xparts_device(inbox.data_ptr(), got)
            part.run(flags)
        return got, int(total.item())

    def send(self, outbox_bytes, counts):
        import torch
        dist = self.dist
        dev = outbox_bytes.device
        send_counts = torch.as_tensor(np.asarray(counts, dtype=np.int64), device=dev)
        recv_counts = torch.empty_like(send_counts)
        dist.all_to_all_single(recv_counts, send_counts, group=self.group)
        rc = [int(x) for x in recv_counts.tolist()]
        sc = [int(x) for x in counts]
        B = self.XPART_BYTES
        out = torch.empty(sum(rc) * B, dtype=torch.uint8, device=dev)
        dist.all_to_all_single(out, outbox_bytes[: sum(sc) * B], [r * B for r in rc], [s * B for s in sc],
                               group=self.group)
        return out, sum(rc)
