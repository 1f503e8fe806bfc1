"""Multi-GPU signal exchange: the manager's Poll merge as a collective.

Reference protocol (one fuzzer per GPU here):
  syz-fuzzer/fuzzer.go:358-364   drain newSignal into PollArgs.MaxSignal
  syz-manager/manager.go:949-962 merge into the manager's maxSignal, fan the
                                 new part out to every other fuzzer
  syz-fuzzer/fuzzer.go:392-398   add the received signal to the local maxSignal
Every rank's maxSignal therefore gains the union of all ranks' newSignal.
Signal sets are 2^32-bit bitmaps, so the union is a bitwise OR of the
newSignal bitmaps.  RCCL (and gloo) have no bitwise-OR reduction, so it is
built from an all-to-all of 1/N shards, a local OR of the N received shards,
and an all-gather of the OR'd shards: 2*(N-1)/N of the bitmap per rank, fixed
regardless of how much signal is new.
"""
import torch
import torch.distributed as dist


def _all_gather_into(out, shard, group):
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, shard, group=group)
    else:  # gloo: list form
        parts = list(out.view(dist.get_world_size(group), -1).unbind(0))
        dist.all_gather(parts, shard, group=group)


class OrExchange:
    """Bitwise-OR all-reduce of an int32 word buffer over the ranks of `group`,
    with buffers allocated once (the bitmap is 512 MiB per rank)."""

    def __init__(self, like, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if self.world > 1:
            if like.numel() % self.world:
                raise ValueError("word count must divide by the world size")
            self.recv = torch.empty_like(like)
            self.full = torch.empty_like(like)

    def __call__(self, words):
        """Returns a tensor holding OR over ranks of `words` (words itself at N=1)."""
        if self.world == 1:
            return words
        dist.all_to_all_single(self.recv, words, group=self.group)
        shards = self.recv.view(self.world, -1)
        acc = shards[0].clone()
        for i in range(1, self.world):
            acc.bitwise_or_(shards[i])
        _all_gather_into(self.full, acc, self.group)
        return self.full


def or_allreduce(words, group=None):
    return OrExchange(words, group)(words).clone()
