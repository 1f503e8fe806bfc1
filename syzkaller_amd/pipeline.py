"""The fuzzer's triage loop (syz-fuzzer/fuzzer.go:645-693) over a stream of
batches, in two overlapped stages.

A batch's triage is its partition (both partition passes, which read only the
batch) and its bucket stage (the new-signal test against maxSignal, the
first-owner flags and the set updates, which must see every earlier batch's
updates).  `PipelinedTriage` queues batch i+1's partition on one stream while
batch i's bucket stage runs on another: the partition kernels are
HBM-bound and the bucket kernel LDS/latency-bound, so the two share the chip.
The bucket stages run in submission order on one stream, so batch i+1 is
tested against maxSignal after batch i, as in the sequential loop.  Two
partition slots of the context (include/syzsig.h sg_prefix_begin_form_dev
form 2) hold batches i and i+1; a slot is re-used after its bucket stage has
finished.  The results equal sg_triage_batch_dev's batch by batch
(tests/test_pipeline.py)."""
import torch

from ._lib import call


class PipelinedTriage:
    def __init__(self, ctx, part_stream=None, bucket_stream=None):
        self.ctx = ctx
        self.sp = part_stream if part_stream is not None else torch.cuda.Stream()
        self.sb = bucket_stream if bucket_stream is not None else torch.cuda.current_stream()
        self.i = 0
        self.end_ev = [None, None]  # per slot: its last bucket stage

    def submit(self, maxset, newset, vals, off, nvals, nrec, rec_new):
        """Queue one batch: flags into rec_new[:nrec] (uint8), maxset/newset
        updated, all on the bucket stream.  vals (int32/uint32 signal) and off
        (int64 record offsets, nrec + 1) must stay unchanged until the
        partition has run (wait on `partition_event`)."""
        slot = self.i & 1
        self.i += 1
        if self.end_ev[slot] is not None:
            self.sp.wait_event(self.end_ev[slot])  # the slot's previous batch is through its bucket stage
        self.ctx.set_stream(self.sp.cuda_stream)
        call("sg_prefix_begin_form_dev", self.ctx.h, slot, 2, None, None, vals.data_ptr() if nvals else None,
             off.data_ptr(), nvals, nrec, None)
        self.partition_event = torch.cuda.Event()
        self.partition_event.record(self.sp)
        self.sb.wait_event(self.partition_event)
        self.ctx.set_stream(self.sb.cuda_stream)
        call("sg_prefix_end_dev", self.ctx.h, slot, maxset.h, None, newset.h if newset is not None else None,
             rec_new.data_ptr() if nrec else None)
        ev = torch.cuda.Event()
        ev.record(self.sb)
        self.end_ev[slot] = ev
        return ev

    def close(self):
        """Queue nothing more; the context's stream goes back to the bucket stream."""
        self.ctx.set_stream(self.sb.cuda_stream)

