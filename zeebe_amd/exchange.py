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
    pms = np.isin(kind, abi.PMS_KINDS)
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
        import torch
        streams = {p.L.zbhip_stream(p.h) for p in self.parts}
        if len(streams) != 1:  # the copies between partitions are ordered by one stream
            raise ValueError("LocalExchange: the partitions must launch on one stream")
        with torch.cuda.stream(self.parts[0].torch_stream()):
            return self._step()

    def _step(self):
        import ctypes as C

        import torch
        from .native import check
        P = len(self.parts)
        mat = torch.zeros((P, P), dtype=torch.int32, device=self.inbox[0].device)
        src = [p.outbox_device_async(mat[s_].data_ptr()) for s_, p in enumerate(self.parts)]
        buckets = mat.cpu().numpy().astype(np.int64)  # one host wait for all of them (the inbox sizes)
        self.sizes = [int(buckets[:, t].sum()) for t in range(P)]
        if buckets.sum():
            # every (source, target) bucket into the targets' inboxes in one launch (zbhip_exchange_gather)
            vp = C.c_void_p * P
            L = self.parts[0].L
            check(L.zbhip_exchange_gather(vp(*src), P, mat.data_ptr(), vp(*[b.data_ptr() for b in self.inbox]),
                                          int(buckets.max()), L.zbhip_stream(self.parts[0].h)), "zbhip_exchange_gather")
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
    partition r + 1), one exchange round per call of :meth:`exchange_partition`:

    1. the partition buckets its outbox by target on the device and copies the per-target counts
       into a device buffer (``zbhip_outbox_device_async``, no host wait);
    2. one ``all_gather`` of the counts: every rank learns the whole P x P send matrix, i.e. its
       receive splits and the global total (the round's termination test) -- the round's only
       host synchronisation;
    3. one ``all_to_all_single`` of the 48-byte commands with those splits.  With the ``nccl``
       backend this is RCCL over xGMI (each GPU pair on its own link, no ring);
    4. the received commands (sources in rank order, each in send order: the order the oracle
       cluster uses) become the partition's next window, built on the device
       (``zbhip_submit_xparts_device``), and run.

    With the ``gloo`` backend (CPU collectives: the multi-process tests, several ranks sharing one
    GPU) the counts and commands are staged through host memory; the partition side is the same.
    """

    XPART_BYTES = abi.XPART_DTYPE.itemsize

    def __init__(self, group=None, max_entries=0, device=None):
        import torch
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.host = dist.get_backend(group) == "gloo"
        self.device = device
        self.max_entries = max_entries
        self.inbox = None
        if max_entries and device is not None:
            self.inbox = torch.empty(max_entries * self.XPART_BYTES, dtype=torch.uint8, device=device)
        self.rounds = 0
        self.sent = 0

    def _inbox(self, n, device):
        import torch
        if self.inbox is None or self.inbox.numel() < n * self.XPART_BYTES:
            self.inbox = torch.empty(max(n, self.max_entries) * self.XPART_BYTES, dtype=torch.uint8, device=device)
        return self.inbox

    def exchange_partition(self, part, staging, flags=0):
        """One exchange round for this rank's partition: send its device outbox, receive its inbox,
        submit and run it.  ``staging`` is a uint8 device tensor of at least the outbox's bytes.
        Returns (received, total sent over all ranks); every rank calls it the same number of
        times, and a round with total 0 ends the exchange."""
        import torch
        if staging.device.type != "cuda":  # host-only partitions (CPU tests)
            return self._exchange(part, staging, flags)
        with torch.cuda.stream(part.torch_stream()):  # ordered with the partition's launches
            return self._exchange(part, staging, flags)

    def _exchange(self, part, staging, flags):
        import torch
        dist, P, B = self.dist, self.world, self.XPART_BYTES
        dev = staging.device
        cnt = torch.zeros(P, dtype=torch.int32, device=dev)
        part.outbox_device_async(cnt.data_ptr())
        if self.host:
            cnt = cnt.cpu()
        rows = [torch.empty_like(cnt) for _ in range(P)]
        dist.all_gather(rows, cnt, group=self.group)
        mat = torch.stack(rows).cpu().numpy().astype(np.int64)  # [source][target]
        total = int(mat.sum())
        if total == 0:
            return 0, 0
        send = [int(x) for x in mat[self.rank]]
        recv = [int(x) for x in mat[:, self.rank]]
        n_send, n_recv = sum(send), sum(recv)
        if n_send:
            part.outbox_copy(staging.data_ptr(), 0, n_send)
        src = staging[: n_send * B]
        if self.host:
            src = src.cpu()
            out = torch.empty(n_recv * B, dtype=torch.uint8)
        else:
            out = self._inbox(n_recv, dev)[: n_recv * B]
        dist.all_to_all_single(out, src, [r * B for r in recv], [s * B for s in send], group=self.group)
        if self.host and n_recv:
            out = self._inbox(n_recv, dev)[: n_recv * B].copy_(out)
        self.rounds += 1
        self.sent += n_send
        if n_recv:
            part.submit_xparts_device(out.data_ptr(), n_recv)
            part.run(flags)
        return n_recv, total

    def send(self, outbox_bytes, counts):
        """Host-driven form (CPU tests): ``outbox_bytes`` already bucketed by target, ``counts`` per
        target; returns the received bucket concatenation and its length."""
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
