#!/usr/bin/env python3
"""Known-byte kernels for calibrating FETCH_SIZE / WRITE_SIZE on gfx950
(MI355X_MICROARCH.md §HBM: calibrate on a known byte count in your own access
pattern).  Run under rocprofv3 --pmc in the same passes as the bench:
  stream : sum of a 4 GiB int32 tensor            -> 4 GiB read, wide coalesced
  gather : 512 MiB int32 table, 256M random 4-B gathers (+1 GiB int32 index read)
  scatter: 256M random 4-B stores into the table (+index/value reads)
Prints the byte counts to compare with the counters."""
import torch

torch.cuda.set_device(0)
n = 1 << 30
x = torch.ones(n, dtype=torch.int32, device="cuda")
s = x.sum()
table = torch.zeros(1 << 27, dtype=torch.int32, device="cuda")  # 512 MiB like a signal bitmap
idx = torch.randint(0, 1 << 27, (1 << 28,), dtype=torch.int64, device="cuda").to(torch.int32)
g = table[idx]  # gather: 256M random 4-B reads
table[idx] = g  # scatter: 256M random 4-B writes
torch.cuda.synchronize()
print({"stream_read_bytes": n * 4, "gather_count": 1 << 28, "table_bytes": 1 << 29, "idx_bytes": (1 << 28) * 4,
       "sum": int(s)})
