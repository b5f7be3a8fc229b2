#!/usr/bin/env python3
"""Device->host transfer costs for result-sized arrays (pinned alloc, copy, sync)."""
import time

import torch


def t(f, n=20):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a = time.perf_counter()
        f()
        ts.append((time.perf_counter() - a) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda")
    R = 1_130_000
    arrs = [torch.randint(0, 1000, (R,), dtype=torch.int32, device=dev),
            torch.randint(0, 1000, (R,), dtype=torch.int16, device=dev),
            torch.randn(1, R, dtype=torch.float64, device=dev)]
    total = sum(a.numel() * a.element_size() for a in arrs)
    print(f"{len(arrs)} arrays, {total / 1e6:.1f} MB")

    def pinned_each():
        outs = []
        for a in arrs:
            h = torch.empty(a.shape, dtype=a.dtype, pin_memory=True)
            h.copy_(a, non_blocking=True)
            outs.append(h)
        torch.cuda.current_stream().synchronize()
        return outs

    pre = [torch.empty(a.shape, dtype=a.dtype, pin_memory=True) for a in arrs]

    def pinned_pre():
        for h, a in zip(pre, arrs):
            h.copy_(a, non_blocking=True)
        torch.cuda.current_stream().synchronize()

    def cpu():
        return [a.cpu() for a in arrs]

    def alloc_only():
        return [torch.empty(a.shape, dtype=a.dtype, pin_memory=True) for a in arrs]

    big = torch.empty(total, dtype=torch.uint8, device=dev)
    bigh = torch.empty(total, dtype=torch.uint8, pin_memory=True)

    def one_copy():
        bigh.copy_(big, non_blocking=True)
        torch.cuda.current_stream().synchronize()

    for name, f in [("pinned alloc + copy each", pinned_each), ("preallocated pinned", pinned_pre),
                    (".cpu()", cpu), ("pinned alloc only", alloc_only), ("one contiguous copy", one_copy)]:
        ms = t(f)
        print(f"{name:28s} {ms:7.3f} ms  {total / ms / 1e6:6.1f} GB/s")


if __name__ == "__main__":
    main()
