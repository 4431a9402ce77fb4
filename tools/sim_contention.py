"""Diagnostic: is the sim's output independent of what runs beside it?
Runs E replicas for STEPS steps twice with the same actions -- alone, then
with a large GEMM running on another stream during every sim launch -- and
reports the first step whose observations differ.  usage: [path] [E]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmdqn_amd.env import EnvConfig, TrafficEnv  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
STEPS = 60
g = torch.Generator(device="cuda").manual_seed(0)
acts = [torch.randint(0, 4, (E, 16), device="cuda", generator=g, dtype=torch.int32)
        for _ in range(STEPS)]
runs = []
KIND = os.environ.get("CONTEND", "gemm")  # gemm | learn | learn_seq (same stream, before)
ag = None
if KIND.startswith("learn"):
    from dmdqn_amd.agent import AgentConfig, BatchedDQN
    ag = BatchedDQN(E, 16, AgentConfig(precision=os.environ.get("PREC", "fp16"), replay_buffer_size=200, seed=1))
    z = torch.zeros((E, 16, 89), device="cuda")
    r = torch.zeros((E, 16), dtype=torch.float64, device="cuda")
    for _ in range(130):
        ag.remember(z, acts[0], r, z, False)
noise = probe = None
if KIND == "noise":
    import ctypes
    noise = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblds_noise.so"))
    sink = torch.zeros(512, dtype=torch.int32, device="cuda")
if KIND == "scratchy":
    import ctypes
    probe = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblds_probe.so"))
    sout = torch.zeros(4096 * 256, device="cuda")
for contended in (False, True):
    env = TrafficEnv(EnvConfig(rows=4, cols=4, num_envs=E, seed=3,
                               step_duration=int(os.environ.get("SUBSTEPS", "10")),
                               cap_lane=int(os.environ.get("CAP", "24"))))
    env.reset()
    side = torch.cuda.Stream()
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.float16)
    out = []
    for t in range(STEPS):
        if contended and KIND == "learn_seq":
            ag.learn()
        elif contended:
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                if probe is not None:
                    probe.scratchy(4096, int(os.environ.get("NOISE_ITERS", "2000")),
                                   ctypes.c_void_p(sout.data_ptr()),
                                   ctypes.c_void_p(side.cuda_stream))
                elif noise is not None:
                    noise.lds_noise(512, int(os.environ.get("NOISE_ITERS", "2000")),
                                    ctypes.c_void_p(sink.data_ptr()),
                                    ctypes.c_void_p(side.cuda_stream))
                elif ag is not None:
                    ag.learn()
                else:
                    for _ in range(3):
                        b = a @ a
        env.step(acts[t])
        out.append([env.obs.clone()] + [x.clone() for x in env._sim_state]
                   + [env.halt.clone(), env.phase.clone(), env.tspent.clone(), env.local.clone()])
    torch.cuda.synchronize()
    runs.append([[x.cpu() for x in o] for o in out])
    del env
first = None
NAMES = ["obs", "x", "v", "dst", "head", "cnt", "req", "gfrom", "fx", "fv", "phase", "ts", "qptr",
         "stats", "last_det", "halt", "phase_out", "tspent", "local"]
for t in range(STEPS):
    for k, (p, q) in enumerate(zip(runs[0][t], runs[1][t])):
        if not torch.equal(p, q):
            m = p != q
            idx = m.nonzero()[:4].tolist()
            if first is None:
                first = (t, NAMES[k], int(m.sum()), idx)
            print("step", t, NAMES[k], int(m.sum()), idx,
                  [(p[tuple(i)].item(), q[tuple(i)].item()) for i in idx])
    if first is not None:
        if first[1] in ("x", "v"):
            e, l = first[3][0][0], first[3][0][1]
            for tt in (t - 1, t):
                if tt < 0:
                    continue
                for r in (0, 1):
                    st = runs[r][tt]
                    h, n = int(st[4][e, l]), int(st[5][e, l])
                    sl = [(h + i) % st[1].shape[2] for i in range(n)]
                    print(f"run{r} step{tt} env{e} lane{l} head{h} cnt{n} req{int(st[6][e, l])} "
                          f"gfrom{int(st[7][e, l])} fx{float(st[8][e, l]):.6f} fv{float(st[9][e, l]):.6f}")
                    print("   x", [round(float(st[1][e, l, k]), 6) for k in sl])
                    print("   v", [round(float(st[2][e, l, k]), 6) for k in sl])
        break
print("cap", os.environ.get("CAP", "24"), os.environ.get("DMDQN_SIM_PATH", "default"), KIND, os.environ.get("PREC", "fp16"), "first divergence under contention:", first)
