"""Diagnostic: k_sim_step duration vs replica count (HIP events on the stream
the sim runs on), 4x4 grid by default, after a 60-step warm-up.  Tells whether
the launch is bound by the number of block rounds (2 env blocks per CU fit
the LDS image) or by per-block latency.
usage: python tools/sim_bench.py [R C E1,E2,...]"""
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from dmdqn_amd.env import EnvConfig, TrafficEnv  # noqa: E402

R, C = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (4, 4)
Es = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [256, 512, 768, 1024, 2048]
for E in Es:
    env = TrafficEnv(EnvConfig(rows=R, cols=C, num_envs=E, seed=3))
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    ms = []
    for step in range(100):
        a = torch.randint(0, 4, (E, env.A), device="cuda", generator=g, dtype=torch.int32)
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        env.step(a)
        s1.record()
        if step >= 60:
            torch.cuda.synchronize()
            ms.append(s0.elapsed_time(s1))
    print(f"{R}x{C} E={E}: step (sim + observe) {np.median(ms):.4f} ms median, "
          f"running {env.stats()[:, 2].mean():.0f}", flush=True)
    del env
    torch.cuda.empty_cache()
