#!/usr/bin/env python3
"""Device-to-host copy rates for the table path's text columns (GBs of uint8):
pageable .cpu(), a fresh pinned buffer (allocation + copy), a reused pinned
buffer, and pageable copies of 8 chunks from 8 threads."""
import json
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

n = int(2.3e9)
t = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
out = {"bytes": n}


def timed(name, f, reps=2):
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    out[name] = {"s": best, "GBps": n / best / 1e9}


timed("pageable", lambda: t.cpu().numpy())
timed("pinned_alloc_only", lambda: torch.empty(n, dtype=torch.uint8, pin_memory=True), reps=1)
h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
timed("pinned_reused_copy", lambda: h.copy_(t, non_blocking=True))


def fresh_pinned():
    x = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    x.copy_(t, non_blocking=True)


timed("pinned_fresh_alloc_copy", fresh_pinned, reps=1)
dst = np.empty(n, np.uint8)
chunks = 8
step = (n + chunks - 1) // chunks


def part(i):
    a, b = i * step, min(n, (i + 1) * step)
    torch.from_numpy(dst[a:b]).copy_(t[a:b])


pool = ThreadPoolExecutor(chunks)
timed("pageable_8_threads", lambda: list(pool.map(part, range(chunks))))
print(json.dumps(out))
