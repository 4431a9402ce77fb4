"""Run tools/pk_hazard.hip's probe (build: hipcc --offload-arch=gfx950 -O3
-shared -fPIC tools/pk_hazard.hip -o tools/libpk_hazard.so) for every mode,
with and without MFMA waves on the same SIMDs; prints the stale-read counts."""
import ctypes
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpk_hazard.so"))
sink = torch.zeros(512, device="cuda")
s = torch.cuda.current_stream()
NAMES = ["mov v->pk_mul", "mov s->pk_mul", "add->pk_mul", "mov s,nop0->pk_mul",
         "mov s,nop1->pk_mul", "mov s->pk_add", "mov s->pk_fma", "mov s(hi)->pk_mul op_sel",
         "mov s->mul (control)", "pk_add,nop0,mov->pk_mul", "pk_add,nop0,mov->mul",
         "pk_add,nop1,mov->pk_mul", "pk_add,nop2,mov->pk_mul", "pk_add,nop1,mov->mul",
         "pk_mul,nop0,mov->mul", "sim sequence verbatim",
         "15, pk_mul no op_sel", "15, pk_add no neg", "15 with s_nop 1", "15 with s_nop 2",
         "15 without the v_mov", "15, v_mov to the high half",
         "pk_mul op_sel_hi:[0,1]", "pk_mul op_sel:[1,0]", "pk_mul op_sel_hi:[1,0]",
         "pk_add op_sel_hi:[0,1]", "pk_add neg_lo/hi:[0,1]", "pk_mul plain", "pk_mul op_sel:[0,1]",
         "pk_fma op_sel_hi:[0,1,1]"]
import struct
f32 = lambda u: struct.unpack("f", struct.pack("I", u & 0xFFFFFFFF))[0]  # noqa: E731
ag = None
if os.environ.get("BESIDE_LEARN"):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dmdqn_amd.agent import AgentConfig, BatchedDQN
    E = 1024
    ag = BatchedDQN(E, 16, AgentConfig(precision="fp16", replay_buffer_size=200, seed=1))
    z = torch.zeros((E, 16, 89), device="cuda")
    r = torch.zeros((E, 16), dtype=torch.float64, device="cuda")
    a = torch.zeros((E, 16), dtype=torch.int32, device="cuda")
    for _ in range(130):
        ag.remember(z, a, r, z, False)
    side = torch.cuda.Stream()
MODES = [int(m) for m in os.environ.get("MODES", "").split(",") if m] or range(len(NAMES))
for mode in MODES:
    name = NAMES[mode]
    row = []
    for mfma in ((0, 1) if ag is None else (2,)):
        err = torch.zeros(3, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        if ag is not None:
            with torch.cuda.stream(side):
                for _ in range(4):
                    ag.learn()
        for _ in range(1 if ag is None else 20):
            lib.pk_probe(1024, 4000 if ag is None else 200, mode, mfma,
                         ctypes.c_void_p(err.data_ptr()), ctypes.c_void_p(sink.data_ptr()),
                         ctypes.c_void_p(s.cuda_stream))
        torch.cuda.synchronize()
        e = err.cpu().tolist()
        row.append(int(e[0]))
        if e[0]:
            print(f"   mode {mode}: a wrong value {f32(e[1])} (lane's old {f32(e[2])}, other 2.0, new 5.0)")
    if ag is None:
        print(f"mode {mode} {name:28s} stale reads: alone {row[0]:8d}  beside MFMA {row[1]:8d}"
              f"  (of {1024 * 256 * 4000} probes)", flush=True)
    else:
        print(f"mode {mode} {name:28s} stale reads beside the fp16 learn: {row[0]:8d}"
              f"  (of {20 * 1024 * 256 * 200} probes)", flush=True)
