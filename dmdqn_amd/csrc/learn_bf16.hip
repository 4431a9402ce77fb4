// learn_bf16.hip -- the bf16 instantiation of learn_h16.hpp: the fused
// per-agent Double-DQN learn (dqn_agent.py:328-380) with bf16 MFMA operands
// (v_mfma_f32_16x16x32_bf16), f32 accumulation, f32 master weights + Adam --
// a mixed_bfloat16 policy (BASELINE config C2).  Precision 2 of dmdqn_learn.
#define DMDQN_H16_BF16 1
#include "learn_h16.hpp"
