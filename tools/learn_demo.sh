#!/bin/bash
# End-to-end check of the whole loop: the batched train.py on the shipped 3x3
# scenario (1024 replicas, fp16, epsilon 1 throughout as on the reference's
# training path, EPISODES episodes; the reference trains 100), the junction
# nets of replica 0 exported in the reference's per-junction naming, then
# src/scripts/test.py: greedy DQN (epsilon 0.01) vs the random policy on
# held-out seeds.  Weights, metrics and the evaluation land in gpurun_out/demo
# (the checkpoint stays on the box).
set -e
O=gpurun_out/demo
W=${TMPDIR:-/tmp}/dmdqn_demo
mkdir -p $O $W
timeout -k 10 900 python src/scripts/train.py --batched --grid 3x3 --envs 1024 --episodes ${EPISODES:-100} \
    --scenario config/scenarios/grid_3x3_p06.npz --save_dir $W --metrics $O/metrics.jsonl \
    --log_every 240 > $O/train.log 2>&1
tail -2 $O/train.log
cp $W/agent_*.weights.npz $O/
timeout -k 10 600 python src/scripts/test.py --model_dir $O --num_eval_episodes 5 --modes dqn random \
    --output_csv $O/eval.csv > $O/eval.log 2>&1
tail -12 $O/eval.log
