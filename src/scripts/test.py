"""src/scripts/test.py -- evaluation of trained agents vs baselines (drop-in for
the reference's src/scripts/test.py:23-259) on the GPU path.

Same arguments and outputs: per-episode rows (mode, seed, total_reward,
avg_reward_per_agent, avg_step_queue_sum, steps) to --output_csv and the
per-mode summary (mean/std reward and queue, mean steps, episodes).  Every
evaluation episode of a mode runs as one env replica (dmdqn_amd/evaluate.py).

--model_dir holds agent_<J_r_c>.weights.npz files (DQNAgent.save_model /
dmdqn_amd.checkpoint.export_keras_weights; the reference's .h5 needs HDF5,
which is absent), or pass --checkpoint (a dmdqn_amd.checkpoint file) to take
the nets of env replica 0.
"""
import argparse
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

import yaml  # noqa: E402

from dmdqn_amd import evaluate as EV  # noqa: E402
from dmdqn_amd.agent import AgentConfig, kernel_to_keras, n_params  # noqa: E402
from dmdqn_amd.checkpoint import load_keras_weights  # noqa: E402
from dmdqn_amd.env import EnvConfig  # noqa: E402
from dmdqn_amd.scenario import Grid  # noqa: E402

DEFAULT_SCENARIO = os.path.join(_ROOT, "config", "scenarios", "grid_3x3_p06.npz")


def parse_eval_args(argv=None):
    p = argparse.ArgumentParser(description="Evaluate MARL Traffic Agents")
    p.add_argument("--agent_config", default=os.path.join(_ROOT, "config", "agent_config.yaml"))
    p.add_argument("--env_config", default=None, help="unused here (kept for the reference CLI)")
    p.add_argument("--model_dir", default=None)
    p.add_argument("--checkpoint", default=None)
    p.add_argument("--num_eval_episodes", type=int, default=10)
    p.add_argument("--eval_seed_start", type=int, default=10000)
    p.add_argument("--eval_epsilon", type=float, default=0.01)
    p.add_argument("--modes", nargs="+", default=["dqn", "random"])
    p.add_argument("--output_csv", default="evaluation_results.csv")
    p.add_argument("--scenario", default=DEFAULT_SCENARIO,
                   help="SUMO scenario (.sumocfg or .npz) or 'synthetic' with --grid")
    p.add_argument("--grid", default="3x3")
    p.add_argument("--max_steps_per_episode", type=int, default=1000)
    p.add_argument("--actuated", action="store_true",
                   help="SUMO's actuated gap-out on phase 0 (grid_3x3.net.xml:894; default fixed)")
    return p.parse_args(argv)


def _weights(args, grid):
    if args.checkpoint:
        import torch
        st = torch.load(args.checkpoint, map_location="cpu", weights_only=True)
        P = st["agent"]["params"].numpy()     # kernel layout [NA or 1, P]
        H = next(h for h in (64, 128) if n_params(h) == P.shape[1])
        return kernel_to_keras(P[:grid.A] if P.shape[0] > 1 else P, H)  # env replica 0
    ws = []
    for jid in grid.junction_ids:
        path = os.path.join(args.model_dir, f"agent_{jid}.weights.npz")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} (train with --save_dir, or export_keras_weights)")
        ws.append(load_keras_weights(path))
    return ws


def main_eval(argv=None):
    args = parse_eval_args(argv)
    modes = list(args.modes)
    scenario = None if args.scenario == "synthetic" else args.scenario
    rows, cols = (int(x) for x in args.grid.split("x"))
    env_cfg = EnvConfig(rows=rows, cols=cols, scenario=scenario, actuated=args.actuated)
    if scenario:
        from dmdqn_amd.sumo_scenario import load_scenario
        sc = load_scenario(scenario)
        rows, cols = sc.rows, sc.cols
    grid = Grid(rows, cols)
    acfg = AgentConfig()
    if os.path.exists(args.agent_config):
        with open(args.agent_config) as f:
            acfg = AgentConfig.from_dict(yaml.safe_load(f) or {})
    acfg.precision = "fp32"
    weights = None
    if "dqn" in modes:
        if not (args.model_dir or args.checkpoint):
            print("Error: --model_dir / --checkpoint not given. Cannot evaluate DQN mode.")
            modes.remove("dqn")
        else:
            weights = _weights(args, grid)
    rows_out = EV.evaluate(env_cfg, modes, args.num_eval_episodes, args.eval_seed_start,
                           args.eval_epsilon, weights, acfg, args.max_steps_per_episode)
    summary = EV.summarize(rows_out)
    print("\n--- Evaluation Summary ---")
    print(summary)
    import pandas as pd
    pd.DataFrame(rows_out).to_csv(args.output_csv, index=False)
    print(f"\nDetailed evaluation results saved to: {args.output_csv}")
    return rows_out, summary


if __name__ == "__main__":
    main_eval()
