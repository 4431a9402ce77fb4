import sys, numpy as np, torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import test_gpu_learn as T
from dmdqn_amd.agent import AgentConfig, BatchedDQN
O = T.O
cfg = AgentConfig(replay_buffer_size=300, target_update_frequency=2, seed=5, precision="fp16")
ag = BatchedDQN(2, 4, cfg)
rng = np.random.RandomState(2)
T._fill(ag, 200, rng)
p0 = ag.keras_params("params").copy(); t0 = ag.keras_params("target").copy()
loss = ag.learn().cpu().numpy(); idx = ag.idx.cpu().numpy()
m_g = ag.keras_params("adam_m")
H = 128
names = [("W1", 89*H), ("b1", H), ("W2", H*H), ("b2", H), ("W3", H*4), ("b3", 4)]
for j in range(2):
    S, Aa, Rn, S2, D = T._host_batch(ag, j, idx[j])
    z = np.zeros_like(p0[j])
    l_e, g_e, *_ = T._mixed_emulation(p0[j], t0[j], z, z.copy(), S, Aa, Rn, S2, D, 1)
    g_g = m_g[j] / np.float32(0.1)
    gs = np.abs(g_e).max()
    bad = ~(np.abs(g_g - g_e) <= 2e-3 * gs + 1e-2 * np.abs(g_e))
    o = 0
    for nm, n in names:
        b = bad[o:o+n]
        print(j, nm, int(b.sum()), "maxabs", float(np.abs(g_g[o:o+n]-g_e[o:o+n]).max()), "scale", float(np.abs(g_e[o:o+n]).max()))
        if nm in ("W2", "W1") and b.sum():
            ii = np.nonzero(b)[0][:10]
            r, c = np.unravel_index(ii, (89 if nm=="W1" else H, H))
            print("   rows", r, "cols", c, g_g[o+ii], g_e[o+ii])
        o += n
