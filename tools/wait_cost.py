"""Diagnostic: what a cross-stream wait costs between back-to-back kernels on
one stream.  Stream A runs N spin kernels (torch.cuda._sleep) of ~200 us;
variants: plain; each preceded by A waiting on an event recorded on an idle
stream B (already complete); A recording an event after each (or every 4th)
kernel that B waits on; the same with CU-masked streams (the bench's
--cu-split layout: A on 192 CUs, B on 64).  Prints the mean time per kernel
(us) of each variant, and the extra per kernel over the plain run.  usage: python tools/wait_cost.py [N]"""
import json
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from dmdqn_amd._lib import cu_masked_stream  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100
dev = torch.device("cuda", 0)
CYC = 200 * 2100  # ~200 us at ~2.1 GHz


def run_rev(a, b, every=1):
    """A records an event after each kernel; B waits on it (every `every`-th
    kernel) and runs a tiny kernel: the cost on A of being waited on."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(a):
        torch.cuda._sleep(20 * CYC)
    for k in range(N):
        with torch.cuda.stream(a):
            torch.cuda._sleep(CYC)
        if k % every == 0:
            ev = torch.cuda.Event()
            ev.record(a)
            b.wait_event(ev)
            with torch.cuda.stream(b):
                torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def run(a, b, wait, tiny_on_b=False):
    torch.cuda.synchronize()
    with torch.cuda.stream(a):
        torch.cuda._sleep(CYC)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(a):
        torch.cuda._sleep(20 * CYC)  # the host queues everything behind this
    for _ in range(N):
        if wait:
            ev = torch.cuda.Event()
            if tiny_on_b:
                with torch.cuda.stream(b):
                    torch.cuda._sleep(1000)
            ev.record(b)
            a.wait_event(ev)
        with torch.cuda.stream(a):
            torch.cuda._sleep(CYC)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return el


out = {}
n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
for name, (a, b) in {"plain": (torch.cuda.Stream(dev), torch.cuda.Stream(dev)),
                     "cumask": (cu_masked_stream(range(64, n_cu), dev),
                                cu_masked_stream(range(64), dev))}.items():
    base = run(a, b, False)
    w = run(a, b, True)
    wk = run(a, b, True, tiny_on_b=True)
    r1, r4 = run_rev(a, b, 1), run_rev(a, b, 4)
    out[name] = {"per_kernel_us": round((base / (N + 20)) * 1e6, 2),
                 "wait_extra_us": round((w - base) / N * 1e6, 2),
                 "wait_on_busy_b_extra_us": round((wk - base) / N * 1e6, 2),
                 "waited_on_by_b_extra_us": round((r1 - base) / N * 1e6, 2),
                 "waited_on_every_4th_extra_us": round((r4 - base) / N * 1e6, 2)}
print(json.dumps(out))
