#!/usr/bin/env python3
"""Profiling-only: how long device allocations take depending on what the memory held before.

    python tools/vram_clear_probe.py alloc GB     # time torch.empty in 8-GiB chunks up to GB, then free and
                                                  # allocate the same again in this process
    python tools/vram_clear_probe.py dirty GB     # allocate GB, write every byte, exit

The question (round-5 VERDICT Weak 5): does a large allocation cost more when the physical pages were used
(written) before -- by an earlier process or earlier in this one -- than on a fresh device?  Each chunk's
time is the hipMalloc behind torch.empty plus a synchronize; the driver clears pages it hands out, and
pages a previous owner wrote may need that clear while untouched ones may not."""
import sys
import time

import torch

CHUNK = 8 << 30


def alloc(total_gb: float, label: str):
    bufs, t_all = [], time.perf_counter()
    times = []
    left = int(total_gb * (1 << 30))
    while left > 0:
        n = min(CHUNK, left)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        bufs.append(torch.empty(n, dtype=torch.uint8, device="cuda"))
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        left -= n
    el = time.perf_counter() - t_all
    print(f"{label}: {total_gb:.0f} GiB in {len(times)} chunks, {el:.3f} s = {total_gb / el:.1f} GiB/s; "
          f"per chunk s: {' '.join(f'{t:.3f}' for t in times)}", flush=True)
    return bufs


def main():
    mode, gb = sys.argv[1], float(sys.argv[2])
    if mode == "dirty":
        bufs = alloc(gb, "dirty-alloc")
        t0 = time.perf_counter()
        for b in bufs:
            b.fill_(0x5A)
        torch.cuda.synchronize()
        print(f"dirty-write: {gb:.0f} GiB in {time.perf_counter() - t0:.3f} s", flush=True)
        return
    bufs = alloc(gb, "first")
    for b in bufs:
        b.fill_(0x33)
    torch.cuda.synchronize()
    del bufs
    torch.cuda.empty_cache()
    torch.cuda.synchronize()
    bufs = alloc(gb, "again-after-free-in-process")
    del bufs
    torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
