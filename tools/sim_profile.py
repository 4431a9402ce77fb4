"""Diagnostic (needs a DMDQN_SIM_PROFILE build): per-pass time of k_sim_step,
thread 0's view, averaged over envs and steps, in microseconds."""
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from dmdqn_amd.env import EnvConfig, TrafficEnv  # noqa: E402

args = [x for x in sys.argv[1:] if not x.startswith("--")]
R, C, E = (int(args[0]), int(args[1]), int(args[2])) if len(args) > 2 else (4, 4, 1024)
fused = "--fused" in sys.argv  # the fused env step (act prologue, observe + store epilogue)
env = TrafficEnv(EnvConfig(rows=R, cols=C, num_envs=E, seed=3))
obs = env.reset()
if fused:
    from dmdqn_amd.agent import AgentConfig, BatchedDQN  # noqa: E402
    ag = BatchedDQN(E, env.A, AgentConfig(replay_buffer_size=200), env_seeds=env.seeds)
g = torch.Generator(device="cuda").manual_seed(0)
acc = np.zeros(10)
n = 0
for step in range(120):
    if fused:
        eps, greedy, out = ag.act_inputs(obs)
        obs = env.step_fused(ag.np_state, eps, greedy, out, ag.ring, obs)[0]
        ag.ring.advance()
    else:
        a = torch.randint(0, 4, (E, env.A), device="cuda", generator=g, dtype=torch.int32)
        env.step(a)
    if step >= 60:
        acc += env.halt.reshape(E, -1)[:, :10].double().mean(0).cpu().numpy() / 100.0
        n += 1
names = ["TL (reg path: prologue to staged vehicles, inside staging)", "A front decide", "B grant", "C advance", "D append", "E insert", "staging",
         "halt+writeback (+ fused epilogue)", "(reg path) start to topology", "(reg path) start to lane order"]
print({k: round(v / n, 2) for k, v in zip(names, acc)}, "us per launch (substep passes summed over K)")
