// dmdqn_torch.cpp -- the C ABI (include/dmdqn.h) registered as PyTorch custom
// operators, torch.ops.dmdqn.* ("Native (TORCH_LIBRARY(dmdqn))").
//
// Every op is a thin, allocation-free adapter: it checks device / dtype /
// contiguity / shape with TORCH_CHECK (a Python RuntimeError), takes the
// current HIP stream of the tensors' device and calls the same extern "C"
// entry point as the ctypes binding.  Ops mutate the arguments their schema
// marks (a!), return nothing, and are registered for the CUDA dispatch key
// (HIP tensors on ROCm) plus a Meta kernel (shape-only, no launch), so the
// dispatcher, torch.compile's fake-tensor tracing and HIP-graph capture see
// them like any other op.  There is no CPU kernel: a CPU tensor raises.
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "../../include/dmdqn.h"

using at::Tensor;
using OptT = std::optional<Tensor>;

namespace {

void *stream_of(const Tensor &t) {
    return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

void check(int rc, const char *what) {
    TORCH_CHECK(rc == DMDQN_OK, what, " failed (rc=", rc, "): ", dmdqn_last_error());
}

template <typename P>
P *dptr(const Tensor &t, at::ScalarType st, const char *name, int64_t numel = -1) {
    TORCH_CHECK(t.is_cuda(), name, " must be a device tensor");
    TORCH_CHECK(t.scalar_type() == st, name, " must be ", st, ", got ", t.scalar_type());
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
    TORCH_CHECK(numel < 0 || t.numel() == numel, name, " has ", t.numel(), " elements, expected ",
                numel);
    return reinterpret_cast<P *>(t.data_ptr());
}

template <typename P>
P *optr(const OptT &t, at::ScalarType st, const char *name, int64_t numel = -1) {
    return t.has_value() ? dptr<P>(*t, st, name, numel) : nullptr;
}

// a 16-bit shadow (f16 or bf16) as raw uint16 storage.  precision (1 = f16,
// 2 = bf16; -1 = either) must match the dtype, so bf16 bits never land in an
// f16 tensor; min_numel > 0 checks the size (NW * Ph, Ph >= P).
uint16_t *h16ptr(const OptT &t, const char *name, int64_t precision = -1, int64_t min_numel = 0) {
    if (!t.has_value()) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kHalf || t->scalar_type() == at::kBFloat16, name,
                " must be float16 or bfloat16");
    TORCH_CHECK(precision < 0 || (precision == 1 && t->scalar_type() == at::kHalf) ||
                    (precision == 2 && t->scalar_type() == at::kBFloat16),
                name, " dtype ", t->scalar_type(), " does not match precision ", precision,
                " (1 = float16, 2 = bfloat16)");
    TORCH_CHECK(t->numel() >= min_numel, name, " holds ", t->numel(), " elements, needs ",
                min_numel);
    TORCH_CHECK(t->is_cuda() && t->is_contiguous(), name, " must be a contiguous device tensor");
    return reinterpret_cast<uint16_t *>(t->data_ptr());
}

int int32_of(int64_t v, const char *name) {
    TORCH_CHECK(v >= INT32_MIN && v <= INT32_MAX, name, " out of int32 range");
    return static_cast<int>(v);
}

constexpr int64_t MT = DMDQN_MT_WORDS;

// ---------------------------------------------------------------- streams / act
void mt_seed(Tensor &state, const Tensor &seeds, const std::string &kind) {
    const int64_t E = seeds.numel();
    auto s = dptr<uint32_t>(state, at::kInt, "state", E * MT);
    auto sd = dptr<uint64_t>(seeds, at::kLong, "seeds");
    c10::hip::HIPGuardMasqueradingAsCUDA g(state.device());
    TORCH_CHECK(kind == "np" || kind == "py", "kind must be 'np' or 'py'");
    check(kind == "np" ? dmdqn_mt_seed_np(s, sd, (int)E, stream_of(state))
                       : dmdqn_mt_seed_py(s, sd, (int)E, stream_of(state)),
          "dmdqn_mt_seed");
}

void mt_draw_u32(Tensor &state, int64_t count, Tensor &out) {
    const int64_t E = state.numel() / MT;
    auto s = dptr<uint32_t>(state, at::kInt, "state", E * MT);
    auto o = dptr<uint32_t>(out, at::kInt, "out", E * count);
    c10::hip::HIPGuardMasqueradingAsCUDA g(state.device());
    check(dmdqn_mt_draw_u32(s, (int)E, int32_of(count, "count"), o, stream_of(state)),
          "dmdqn_mt_draw_u32");
}

void act(Tensor &np_state, int64_t A, double eps, int64_t n_actions, const OptT &greedy,
         Tensor &actions, bool uniform) {
    const int64_t E = np_state.numel() / MT;
    auto s = dptr<uint32_t>(np_state, at::kInt, "np_state", E * MT);
    auto gr = optr<int32_t>(greedy, at::kInt, "greedy", E * A);
    auto out = dptr<int32_t>(actions, at::kInt, "actions", E * A);
    c10::hip::HIPGuardMasqueradingAsCUDA g(np_state.device());
    if (uniform)
        check(dmdqn_act_uniform(s, (int)E, int32_of(A, "A"), int32_of(n_actions, "n_actions"), out,
                                stream_of(np_state)),
              "dmdqn_act_uniform");
    else
        check(dmdqn_act(s, (int)E, int32_of(A, "A"), eps, int32_of(n_actions, "n_actions"), gr, out,
                        stream_of(np_state)),
              "dmdqn_act");
}

// ---------------------------------------------------------------- observe
void observe(int64_t R, int64_t C, const Tensor &halt, const Tensor &phase, const Tensor &tspent,
             int64_t mode, const OptT &local, const OptT &obs, const OptT &prev_local,
             const OptT &reward) {
    const int64_t A = R * C;
    TORCH_CHECK(A > 0 && halt.numel() % (A * 12) == 0, "halt must be [E, R*C, 12]");
    const int64_t E = halt.numel() / (A * 12);
    auto h = dptr<int32_t>(halt, at::kInt, "halt");
    auto p = dptr<int32_t>(phase, at::kInt, "phase", E * A);
    auto ts = dptr<int32_t>(tspent, at::kInt, "tspent", E * A);
    auto lo = optr<float>(local, at::kFloat, "local", E * A * DMDQN_LOCAL_DIM);
    auto ob = optr<float>(obs, at::kFloat, "obs", E * A * DMDQN_OBS_DIM);
    auto pl = optr<float>(prev_local, at::kFloat, "prev_local", E * A * DMDQN_LOCAL_DIM);
    auto rw = optr<double>(reward, at::kDouble, "reward", E * A);
    TORCH_CHECK((pl == nullptr) == (rw == nullptr), "prev_local and reward go together");
    c10::hip::HIPGuardMasqueradingAsCUDA g(halt.device());
    check(dmdqn_observe((int)R, (int)C, (int)E, h, p, ts, (int)mode, lo, ob, pl, rw,
                        stream_of(halt)),
          "dmdqn_observe");
}

// ---------------------------------------------------------------- replay
void replay_store(int64_t slot, const Tensor &obs_s, const Tensor &obs_n, const Tensor &act_,
                  const Tensor &rew, const Tensor &done, Tensor &ring_s, Tensor &ring_n,
                  Tensor &ring_a, Tensor &ring_r, Tensor &ring_d, Tensor &err) {
    const int64_t NA = act_.numel();
    TORCH_CHECK(NA > 0 && ring_a.numel() % NA == 0, "ring_a must be [NA, cap]");
    const int64_t cap = ring_a.numel() / NA;
    auto s = dptr<float>(obs_s, at::kFloat, "obs_s", NA * DMDQN_OBS_DIM);
    auto n = dptr<float>(obs_n, at::kFloat, "obs_n", NA * DMDQN_OBS_DIM);
    auto a = dptr<int32_t>(act_, at::kInt, "act");
    auto r = dptr<double>(rew, at::kDouble, "rew", NA);
    auto d = dptr<uint8_t>(done, at::kByte, "done", NA);
    auto rs = dptr<int8_t>(ring_s, at::kChar, "ring_s", NA * cap * DMDQN_ROW_BYTES);
    auto rn = dptr<int8_t>(ring_n, at::kChar, "ring_n", NA * cap * DMDQN_ROW_BYTES);
    auto ra = dptr<uint8_t>(ring_a, at::kByte, "ring_a", NA * cap);
    auto rr = dptr<double>(ring_r, at::kDouble, "ring_r", NA * cap);
    auto rd = dptr<uint8_t>(ring_d, at::kByte, "ring_d", NA * cap);
    // err: a device tensor, or pinned host memory the kernel writes directly
    TORCH_CHECK(err.is_cuda() || err.is_pinned(), "err must be a device tensor or pinned host memory");
    TORCH_CHECK(err.scalar_type() == at::kInt && err.numel() == 1, "err must be one int32");
    auto e = reinterpret_cast<int32_t *>(err.data_ptr());
    c10::hip::HIPGuardMasqueradingAsCUDA g(obs_s.device());
    check(dmdqn_replay_store((int)NA, int32_of(cap, "cap"), int32_of(slot, "slot"), s, n, a, r, d,
                             rs, rn, ra, rr, rd, e, stream_of(obs_s)),
          "dmdqn_replay_store");
}

void replay_store_f32(int64_t slot, const Tensor &obs_s, const Tensor &obs_n, const Tensor &act_,
                      const Tensor &rew, const Tensor &done, Tensor &rows_s, Tensor &rows_n,
                      Tensor &ring_a, Tensor &ring_r, Tensor &ring_d) {
    const int64_t NA = act_.numel();
    TORCH_CHECK(NA > 0 && ring_a.numel() % NA == 0, "ring_a must be [NA, cap]");
    const int64_t cap = ring_a.numel() / NA;
    auto s = dptr<float>(obs_s, at::kFloat, "obs_s", NA * DMDQN_OBS_DIM);
    auto n = dptr<float>(obs_n, at::kFloat, "obs_n", NA * DMDQN_OBS_DIM);
    auto a = dptr<int32_t>(act_, at::kInt, "act", NA);
    auto r = dptr<double>(rew, at::kDouble, "rew", NA);
    auto d = dptr<uint8_t>(done, at::kByte, "done", NA);
    auto rs = dptr<float>(rows_s, at::kFloat, "rows_s", NA * cap * DMDQN_ROW_FLOATS);
    auto rn = dptr<float>(rows_n, at::kFloat, "rows_n", NA * cap * DMDQN_ROW_FLOATS);
    auto ra = dptr<uint8_t>(ring_a, at::kByte, "ring_a", NA * cap);
    auto rr = dptr<double>(ring_r, at::kDouble, "ring_r", NA * cap);
    auto rd = dptr<uint8_t>(ring_d, at::kByte, "ring_d", NA * cap);
    c10::hip::HIPGuardMasqueradingAsCUDA g(obs_s.device());
    check(dmdqn_replay_store_f32((int)NA, int32_of(cap, "cap"), int32_of(slot, "slot"), s, n, a, r,
                                 d, rs, rn, ra, rr, rd, stream_of(obs_s)),
          "dmdqn_replay_store_f32");
}

void replay_gather_f32(const Tensor &rows_s, const Tensor &rows_n, const Tensor &idx,
                       int64_t start, Tensor &xs, Tensor &xn) {
    TORCH_CHECK(idx.dim() == 2, "idx must be [NA, batch]");
    const int64_t NA = idx.size(0), B = idx.size(1);
    TORCH_CHECK(rows_s.dim() == 3 && rows_s.size(0) == NA && rows_s.size(2) == DMDQN_ROW_FLOATS,
                "rows_s must be [NA, cap, ", DMDQN_ROW_FLOATS, "]");
    const int64_t cap = rows_s.size(1);
    auto rs = dptr<float>(rows_s, at::kFloat, "rows_s", NA * cap * DMDQN_ROW_FLOATS);
    auto rn = dptr<float>(rows_n, at::kFloat, "rows_n", NA * cap * DMDQN_ROW_FLOATS);
    auto ix = dptr<int32_t>(idx, at::kInt, "idx", NA * B);
    auto ps = dptr<float>(xs, at::kFloat, "xs", NA * B * DMDQN_ROW_FLOATS);
    auto pn = dptr<float>(xn, at::kFloat, "xn", NA * B * DMDQN_ROW_FLOATS);
    c10::hip::HIPGuardMasqueradingAsCUDA g(rows_s.device());
    check(dmdqn_replay_gather_f32(rs, rn, ix, (int)NA, int32_of(cap, "cap"), int32_of(start, "start"),
                                  (int)B, ps, pn, stream_of(rows_s)),
          "dmdqn_replay_gather_f32");
}

void replay_sample(Tensor &py_state, int64_t A, int64_t n, int64_t k, Tensor &idx,
                   int64_t lds_budget) {
    const int64_t E = py_state.numel() / MT;
    auto s = dptr<uint32_t>(py_state, at::kInt, "py_state", E * MT);
    auto o = dptr<int32_t>(idx, at::kInt, "idx", E * A * k);
    TORCH_CHECK(lds_budget >= 0, "lds_budget must be >= 0");
    c10::hip::HIPGuardMasqueradingAsCUDA g(py_state.device());
    check(dmdqn_replay_sample_budget(s, (int)E, int32_of(A, "A"), int32_of(n, "n"),
                                     int32_of(k, "k"), (size_t)lds_budget, o, stream_of(py_state)),
          "dmdqn_replay_sample");
}

// ---------------------------------------------------------------- simulator
// state (mutable, in order): x, v, dst, head, cnt, req, gfrom, fx, fv, tl_phase,
// tl_ts, qptr, stats, last_det[, t_env]; tables: q_off, q_ids, vdst, exit_id,
// exit_ao, q_dst; dims: R, C, E, cap_lane, period_ms, nveh, actuated.
dmdqn_sim make_sim(at::TensorList state, at::TensorList tables, at::IntArrayRef dims) {
    TORCH_CHECK((state.size() == 14 || state.size() == 15) && tables.size() == 6 && dims.size() == 7,
                "sim: 14 state tensors (+ t_env), 6 tables, 7 dims");
    dmdqn_sim s{};
    s.R = (int)dims[0]; s.C = (int)dims[1]; s.E = (int)dims[2]; s.cap_lane = (int)dims[3];
    s.period_ms = (int)dims[4]; s.nveh = (int)dims[5]; s.actuated = (int)dims[6];
    const int64_t A = (int64_t)s.R * s.C, X = 2 * (int64_t)s.R + 2 * s.C, E = s.E;
    const int64_t NL = 3 * (4 * A + X), ns = E * NL * s.cap_lane;
    s.x = dptr<float>(state[0], at::kFloat, "x", ns);
    s.v = dptr<float>(state[1], at::kFloat, "v", ns);
    s.dst = dptr<int32_t>(state[2], at::kInt, "dst", ns);
    s.head = dptr<int32_t>(state[3], at::kInt, "head", E * NL);
    s.cnt = dptr<int32_t>(state[4], at::kInt, "cnt", E * NL);
    s.req = dptr<int32_t>(state[5], at::kInt, "req", E * NL);
    s.gfrom = dptr<int32_t>(state[6], at::kInt, "gfrom", E * NL);
    s.fx = dptr<float>(state[7], at::kFloat, "fx", E * NL);
    s.fv = dptr<float>(state[8], at::kFloat, "fv", E * NL);
    s.tl_phase = dptr<int32_t>(state[9], at::kInt, "tl_phase", E * A);
    s.tl_ts = dptr<int32_t>(state[10], at::kInt, "tl_ts", E * A);
    s.qptr = dptr<int32_t>(state[11], at::kInt, "qptr", E * 4 * A);
    s.stats = dptr<int32_t>(state[12], at::kInt, "stats", E * 4);
    s.last_det = dptr<int32_t>(state[13], at::kInt, "last_det", E * 12 * A);
    s.t_env = state.size() == 15 ? dptr<int32_t>(state[14], at::kInt, "t_env", E) : nullptr;
    s.q_off = dptr<int32_t>(tables[0], at::kInt, "q_off", E * (4 * A + 1));
    s.q_ids = dptr<uint16_t>(tables[1], at::kShort, "q_ids", E * s.nveh);
    s.vdst = dptr<uint16_t>(tables[2], at::kShort, "vdst", E * s.nveh);
    s.exit_id = dptr<int32_t>(tables[3], at::kInt, "exit_id", A * 4);
    s.exit_ao = dptr<int32_t>(tables[4], at::kInt, "exit_ao", X * 2);
    s.q_dst = dptr<uint16_t>(tables[5], at::kShort, "q_dst", E * s.nveh);
    return s;
}

void sim_reset(at::TensorList state, at::TensorList tables, at::IntArrayRef dims,
               const OptT &mask) {
    dmdqn_sim s = make_sim(state, tables, dims);
    auto m = optr<uint8_t>(mask, at::kByte, "mask", s.E);
    c10::hip::HIPGuardMasqueradingAsCUDA g(state[0].device());
    check(dmdqn_sim_reset_envs(&s, m, stream_of(state[0])), "dmdqn_sim_reset_envs");
}

void sim_step(at::TensorList state, at::TensorList tables, at::IntArrayRef dims,
              at::ArrayRef<double> idm, const OptT &actions, int64_t stride, int64_t t0, int64_t K,
              int64_t max_time, Tensor &halt, Tensor &phase, Tensor &tspent, Tensor &done) {
    dmdqn_sim s = make_sim(state, tables, dims);
    TORCH_CHECK(idm.size() == 12, "idm: 12 constants (include/dmdqn.h dmdqn_idm order)");
    dmdqn_idm p{(float)idm[0], (float)idm[1], (float)idm[2], (float)idm[3], (float)idm[4],
                (float)idm[5], (float)idm[6], (float)idm[7], (float)idm[8], (float)idm[9],
                (float)idm[10], (float)idm[11]};
    const int64_t A = (int64_t)s.R * s.C, E = s.E;
    auto a = optr<int32_t>(actions, at::kInt, "actions", E * A);
    auto h = dptr<int32_t>(halt, at::kInt, "halt", E * A * 12);
    auto ph = dptr<int32_t>(phase, at::kInt, "phase", E * A);
    auto ts = dptr<int32_t>(tspent, at::kInt, "tspent", E * A);
    auto d = dptr<uint8_t>(done, at::kByte, "done", E);
    c10::hip::HIPGuardMasqueradingAsCUDA g(halt.device());
    check(dmdqn_sim_step(&s, &p, a, (int)stride, int32_of(t0, "t0"), (int)K,
                         int32_of(max_time, "max_time"), h, ph, ts, d, stream_of(halt)),
          "dmdqn_sim_step");
}

// act + sim_step + observe + replay_store (int8 rows) in one launch per env.
void env_step(at::TensorList state, at::TensorList tables, at::IntArrayRef dims,
              at::ArrayRef<double> idm, int64_t stride, int64_t t0, int64_t K, int64_t max_time,
              Tensor &halt, Tensor &phase, Tensor &tspent, Tensor &done, Tensor &np_state,
              const OptT &greedy, Tensor &actions, double eps, int64_t n_actions, int64_t mode,
              Tensor &local, Tensor &obs, const Tensor &prev_local, Tensor &reward,
              const Tensor &obs_s, int64_t slot, Tensor &ring_s, Tensor &ring_n, Tensor &ring_a,
              Tensor &ring_r, Tensor &ring_d, Tensor &err) {
    dmdqn_sim s = make_sim(state, tables, dims);
    TORCH_CHECK(idm.size() == 12, "idm: 12 constants (include/dmdqn.h dmdqn_idm order)");
    dmdqn_idm p{(float)idm[0], (float)idm[1], (float)idm[2], (float)idm[3], (float)idm[4],
                (float)idm[5], (float)idm[6], (float)idm[7], (float)idm[8], (float)idm[9],
                (float)idm[10], (float)idm[11]};
    const int64_t A = (int64_t)s.R * s.C, E = s.E, NA = E * A;
    auto h = dptr<int32_t>(halt, at::kInt, "halt", E * A * 12);
    auto ph = dptr<int32_t>(phase, at::kInt, "phase", E * A);
    auto ts = dptr<int32_t>(tspent, at::kInt, "tspent", E * A);
    auto d = dptr<uint8_t>(done, at::kByte, "done", E);
    TORCH_CHECK(ring_a.numel() % NA == 0 && ring_a.numel() > 0, "ring_a must be [E*A, cap]");
    const int64_t cap = ring_a.numel() / NA;
    dmdqn_env_fuse f{};
    f.np_state = dptr<uint32_t>(np_state, at::kInt, "np_state", E * MT);
    f.greedy = optr<int32_t>(greedy, at::kInt, "greedy", NA);
    f.actions = dptr<int32_t>(actions, at::kInt, "actions", NA);
    f.eps = eps;
    f.n_actions = int32_of(n_actions, "n_actions");
    f.mode = (int)mode;
    f.local = dptr<float>(local, at::kFloat, "local", NA * DMDQN_LOCAL_DIM);
    f.obs = dptr<float>(obs, at::kFloat, "obs", NA * DMDQN_OBS_DIM);
    f.prev_local = dptr<float>(prev_local, at::kFloat, "prev_local", NA * DMDQN_LOCAL_DIM);
    f.reward = dptr<double>(reward, at::kDouble, "reward", NA);
    f.obs_s = dptr<float>(obs_s, at::kFloat, "obs_s", NA * DMDQN_OBS_DIM);
    f.cap = int32_of(cap, "cap");
    f.slot = int32_of(slot, "slot");
    f.ring_s = dptr<int8_t>(ring_s, at::kChar, "ring_s", NA * cap * DMDQN_ROW_BYTES);
    f.ring_n = dptr<int8_t>(ring_n, at::kChar, "ring_n", NA * cap * DMDQN_ROW_BYTES);
    f.ring_a = dptr<uint8_t>(ring_a, at::kByte, "ring_a", NA * cap);
    f.ring_r = dptr<double>(ring_r, at::kDouble, "ring_r", NA * cap);
    f.ring_d = dptr<uint8_t>(ring_d, at::kByte, "ring_d", NA * cap);
    TORCH_CHECK(err.is_cuda() || err.is_pinned(), "err must be a device tensor or pinned host memory");
    TORCH_CHECK(err.scalar_type() == at::kInt && err.numel() == 1, "err must be one int32");
    f.err = reinterpret_cast<int32_t *>(err.data_ptr());
    c10::hip::HIPGuardMasqueradingAsCUDA g(halt.device());
    check(dmdqn_env_step(&s, &p, &f, (int)stride, int32_of(t0, "t0"), (int)K,
                         int32_of(max_time, "max_time"), h, ph, ts, d, stream_of(halt)),
          "dmdqn_env_step");
}

// ---------------------------------------------------------------- learn
dmdqn_learn_args make_learn(const Tensor &ring_s, const Tensor &ring_n, const Tensor &ring_a,
                            const Tensor &ring_d, const Tensor &ring_r, const Tensor &idx,
                            Tensor &params, const OptT &adam_m, const OptT &adam_v,
                            Tensor &target, const OptT &target_h, const OptT &loss, int64_t start,
                            int64_t hidden, int64_t precision, bool sync, double gamma,
                            double alpha, double c1, double c2, double eps, int64_t loss_kind,
                            const OptT &qstats, const OptT &rn_out, const OptT &params_h,
                            const OptT &stamps, int64_t NA, int64_t NW,
                            const OptT &xs = std::nullopt, const OptT &xn = std::nullopt) {
    dmdqn_learn_args a{};
    TORCH_CHECK(NA > 0 && ring_a.numel() % NA == 0, "ring_a must be [NA, cap]");
    const int64_t cap = ring_a.numel() / NA, B = idx.numel() / NA;
    TORCH_CHECK(NW > 0 && params.numel() % NW == 0, "params must be [NW, P]");
    const int64_t P = params.numel() / NW;
    a.NA = (int)NA; a.cap = int32_of(cap, "cap"); a.start = int32_of(start, "start");
    a.batch = (int)B; a.hidden = (int)hidden; a.precision = (int)precision;
    a.sync_target = sync ? 1 : 0; a.P = (int)P;
    TORCH_CHECK(xs.has_value() == xn.has_value(), "xs and xn go together");
    if (xs.has_value()) {  // float rows: the batch pre-gathered (replay_gather_f32)
        a.row_format = DMDQN_ROWS_F32;
        a.xs = dptr<float>(*xs, at::kFloat, "xs", NA * B * DMDQN_ROW_FLOATS);
        a.xn = dptr<float>(*xn, at::kFloat, "xn", NA * B * DMDQN_ROW_FLOATS);
    } else {
        a.ring_s = dptr<int8_t>(ring_s, at::kChar, "ring_s", NA * cap * DMDQN_ROW_BYTES);
        a.ring_n = dptr<int8_t>(ring_n, at::kChar, "ring_n", NA * cap * DMDQN_ROW_BYTES);
    }
    a.ring_a = dptr<uint8_t>(ring_a, at::kByte, "ring_a", NA * cap);
    a.ring_d = dptr<uint8_t>(ring_d, at::kByte, "ring_d", NA * cap);
    a.ring_r = dptr<double>(ring_r, at::kDouble, "ring_r", NA * cap);
    a.idx = dptr<int32_t>(idx, at::kInt, "idx", NA * B);
    a.params = dptr<float>(params, at::kFloat, "params");
    a.adam_m = optr<float>(adam_m, at::kFloat, "adam_m", NW * P);
    a.adam_v = optr<float>(adam_v, at::kFloat, "adam_v", NW * P);
    a.target = dptr<float>(target, at::kFloat, "target", NW * P);
    // the kernels read NW rows of Ph = P rounded up to 8 halves
    const int64_t Ph = (P + 7) / 8 * 8;
    if (precision == 0) TORCH_CHECK(!target_h.has_value(), "target_h is for precision 1 / 2");
    a.target_h = h16ptr(target_h, "target_h", precision == 0 ? -1 : precision, NW * Ph);
    a.loss = optr<float>(loss, at::kFloat, "loss", NA);
    a.gamma = (float)gamma; a.alpha = (float)alpha; a.c1 = (float)c1; a.c2 = (float)c2;
    a.eps = (float)eps;
    a.stamps = optr<uint64_t>(stamps, at::kLong, "stamps", NA * 16);
    a.qstats = optr<float>(qstats, at::kFloat, "qstats", NA * 6);
    a.params_h = h16ptr(params_h, "params_h", precision == 0 ? -1 : precision, NW * Ph);
    a.loss_kind = (int)loss_kind;
    a.rn_out = optr<float>(rn_out, at::kFloat, "rn_out", NA * B);
    return a;
}

void learn_step(const Tensor &ring_s, const Tensor &ring_n, const Tensor &ring_a,
                const Tensor &ring_d, const Tensor &ring_r, const Tensor &idx, Tensor &params,
                Tensor &adam_m, Tensor &adam_v, Tensor &target, const OptT &target_h, Tensor &loss,
                int64_t start, int64_t hidden, int64_t precision, bool sync, double gamma,
                double alpha, double c1, double c2, double eps, int64_t loss_kind,
                const OptT &qstats, const OptT &rn_out, const OptT &stamps, const OptT &grad,
                const OptT &xs, const OptT &xn) {
    const int64_t NA = loss.numel();
    dmdqn_learn_args a = make_learn(ring_s, ring_n, ring_a, ring_d, ring_r, idx, params, adam_m,
                                    adam_v, target, target_h, loss, start, hidden, precision, sync,
                                    gamma, alpha, c1, c2, eps, loss_kind, qstats, rn_out,
                                    std::nullopt, stamps, NA, NA, xs, xn);
    c10::hip::HIPGuardMasqueradingAsCUDA g(params.device());
    if (grad.has_value()) {  // the split learn: gradient launch, then the Adam launch
        auto gr = dptr<float>(*grad, at::kFloat, "grad", NA * (int64_t)a.P);
        check(dmdqn_learn_grad(&a, gr, stream_of(params)), "dmdqn_learn_grad");
        check(dmdqn_adam_agents(&a, gr, stream_of(params)), "dmdqn_adam_agents");
        return;
    }
    check(dmdqn_learn(&a, stream_of(params)), "dmdqn_learn");
}

void learn_shared_grad(const Tensor &ring_s, const Tensor &ring_n, const Tensor &ring_a,
                       const Tensor &ring_d, const Tensor &ring_r, const Tensor &idx,
                       const Tensor &params, const Tensor &target, const Tensor &target_h,
                       const Tensor &params_h, Tensor &loss, int64_t start, double gamma,
                       int64_t loss_kind, const OptT &qstats, const OptT &rn_out, Tensor &slab,
                       const OptT &grad, double scale, const OptT &work) {
    const int64_t NA = loss.numel();
    Tensor p = params, t = target;  // read-only here: the Adam step is a separate op
    dmdqn_learn_args a = make_learn(ring_s, ring_n, ring_a, ring_d, ring_r, idx, p, std::nullopt,
                                    std::nullopt, t, target_h, loss, start, 128, 1, false, gamma,
                                    0.0, 0.0, 0.0, 0.0, loss_kind, qstats, rn_out, params_h,
                                    std::nullopt, NA, 1);
    TORCH_CHECK(slab.numel() % a.P == 0, "slab must be [n_slabs, P]");
    const int n_slabs = (int)(slab.numel() / a.P);
    auto sl = dptr<float>(slab, at::kFloat, "slab");
    auto gr = optr<float>(grad, at::kFloat, "grad", a.P);  // None: dmdqn_adam_slabs reduces
    auto wk = optr<uint8_t>(work, at::kByte, "work",
                            (int64_t)dmdqn_learn_shared_work_bytes((int)NA));
    c10::hip::HIPGuardMasqueradingAsCUDA g(params.device());
    check(dmdqn_learn_shared_grad(&a, sl, n_slabs, gr, (float)scale, wk, stream_of(params)),
          "dmdqn_learn_shared_grad");
}

void adam(Tensor &params, Tensor &adam_m, Tensor &adam_v, Tensor &target, const OptT &target_h,
          const OptT &params_h, const Tensor &grad, double gscale, double alpha, double c1,
          double c2, double eps, bool sync) {
    const int64_t n = params.numel();
    auto w = dptr<float>(params, at::kFloat, "params");
    auto m = dptr<float>(adam_m, at::kFloat, "adam_m", n);
    auto v = dptr<float>(adam_v, at::kFloat, "adam_v", n);
    auto t = dptr<float>(target, at::kFloat, "target", n);
    auto gr = dptr<float>(grad, at::kFloat, "grad", n);
    c10::hip::HIPGuardMasqueradingAsCUDA g(params.device());
    // k_adam writes f16 shadows (the shared net is fp16-only)
    check(dmdqn_adam(w, m, v, t, h16ptr(target_h, "target_h", 1, n), h16ptr(params_h, "params_h", 1, n), gr,
                     int32_of(n, "n"), (float)gscale, (float)alpha, (float)c1, (float)c2,
                     (float)eps, sync ? 1 : 0, stream_of(params)),
          "dmdqn_adam");
}

void adam_slabs(Tensor &params, Tensor &adam_m, Tensor &adam_v, Tensor &target,
                const OptT &target_h, const OptT &params_h, const Tensor &slab, Tensor &grad,
                double scale, double gscale, double alpha, double c1, double c2, double eps,
                bool sync) {
    const int64_t n = params.numel();
    auto w = dptr<float>(params, at::kFloat, "params");
    auto m = dptr<float>(adam_m, at::kFloat, "adam_m", n);
    auto v = dptr<float>(adam_v, at::kFloat, "adam_v", n);
    auto t = dptr<float>(target, at::kFloat, "target", n);
    auto gr = dptr<float>(grad, at::kFloat, "grad", n);
    TORCH_CHECK(slab.numel() % n == 0, "slab must be [n_slabs, P]");
    auto sl = dptr<float>(slab, at::kFloat, "slab");
    c10::hip::HIPGuardMasqueradingAsCUDA g(params.device());
    check(dmdqn_adam_slabs(w, m, v, t, h16ptr(target_h, "target_h", 1, n),
                           h16ptr(params_h, "params_h", 1, n), sl, int32_of(slab.numel() / n, "n_slabs"),
                           gr, (float)scale, int32_of(n, "n"), (float)gscale, (float)alpha,
                           (float)c1, (float)c2, (float)eps, sync ? 1 : 0, stream_of(params)),
          "dmdqn_adam_slabs");
}

void target_sync(const Tensor &params, Tensor &target, const OptT &target_h, int64_t precision) {
    TORCH_CHECK(params.dim() == 2, "params must be [NW, P]");
    const int64_t NW = params.size(0), P = params.size(1);
    auto p = dptr<float>(params, at::kFloat, "params");
    auto t = dptr<float>(target, at::kFloat, "target", NW * P);
    const int64_t Ph = target_h.has_value() ? target_h->numel() / NW : P;
    TORCH_CHECK(!target_h.has_value() || (target_h->numel() % NW == 0 && Ph >= P),
                "target_h must be [NW, Ph] with Ph >= P");
    c10::hip::HIPGuardMasqueradingAsCUDA g(params.device());
    check(dmdqn_target_sync(p, t, h16ptr(target_h, "target_h", precision), (int)NW, (int)P, (int)Ph,
                            (int)precision, stream_of(params)),
          "dmdqn_target_sync");
}

void q_argmax(const Tensor &params, int64_t hidden, int64_t precision, const Tensor &obs,
              Tensor &out, const OptT &q, bool shared) {
    const int64_t NA = out.numel();
    const int64_t P = shared ? params.numel() : params.numel() / NA;
    auto p = dptr<float>(params, at::kFloat, "params");
    auto o = dptr<float>(obs, at::kFloat, "obs", NA * DMDQN_OBS_DIM);
    auto g = dptr<int32_t>(out, at::kInt, "out", NA);
    auto qq = optr<float>(q, at::kFloat, "q", NA * 4);
    c10::hip::HIPGuardMasqueradingAsCUDA gd(params.device());
    check(shared ? dmdqn_q_argmax_shared(p, (int)NA, (int)P, (int)hidden, (int)precision, o, g, qq,
                                         stream_of(params))
                 : dmdqn_q_argmax(p, (int)NA, (int)P, (int)hidden, (int)precision, o, g, qq,
                                  stream_of(params)),
          "dmdqn_q_argmax");
}

// Meta kernels: the ops only mutate their (a!) arguments, so tracing needs no
// shape function beyond "nothing is returned".
void mt_seed_meta(Tensor &, const Tensor &, const std::string &) {}
void mt_draw_u32_meta(Tensor &, int64_t, Tensor &) {}
void act_meta(Tensor &, int64_t, double, int64_t, const OptT &, Tensor &, bool) {}
void observe_meta(int64_t, int64_t, const Tensor &, const Tensor &, const Tensor &, int64_t,
                  const OptT &, const OptT &, const OptT &, const OptT &) {}
void replay_store_meta(int64_t, const Tensor &, const Tensor &, const Tensor &, const Tensor &,
                       const Tensor &, Tensor &, Tensor &, Tensor &, Tensor &, Tensor &, Tensor &) {}
void replay_sample_meta(Tensor &, int64_t, int64_t, int64_t, Tensor &, int64_t) {}
void replay_store_f32_meta(int64_t, const Tensor &, const Tensor &, const Tensor &, const Tensor &,
                           const Tensor &, Tensor &, Tensor &, Tensor &, Tensor &, Tensor &) {}
void replay_gather_f32_meta(const Tensor &, const Tensor &, const Tensor &, int64_t, Tensor &,
                            Tensor &) {}
void sim_reset_meta(at::TensorList, at::TensorList, at::IntArrayRef, const OptT &) {}
void sim_step_meta(at::TensorList, at::TensorList, at::IntArrayRef, at::ArrayRef<double>,
                   const OptT &, int64_t, int64_t, int64_t, int64_t, Tensor &, Tensor &, Tensor &,
                   Tensor &) {}
void env_step_meta(at::TensorList, at::TensorList, at::IntArrayRef, at::ArrayRef<double>, int64_t,
                   int64_t, int64_t, int64_t, Tensor &, Tensor &, Tensor &, Tensor &, Tensor &,
                   const OptT &, Tensor &, double, int64_t, int64_t, Tensor &, Tensor &,
                   const Tensor &, Tensor &, const Tensor &, int64_t, Tensor &, Tensor &, Tensor &,
                   Tensor &, Tensor &, Tensor &) {}
void learn_step_meta(const Tensor &, const Tensor &, const Tensor &, const Tensor &, const Tensor &,
                     const Tensor &, Tensor &, Tensor &, Tensor &, Tensor &, const OptT &, Tensor &,
                     int64_t, int64_t, int64_t, bool, double, double, double, double, double,
                     int64_t, const OptT &, const OptT &, const OptT &, const OptT &, const OptT &,
                     const OptT &) {}
void learn_shared_grad_meta(const Tensor &, const Tensor &, const Tensor &, const Tensor &,
                            const Tensor &, const Tensor &, const Tensor &, const Tensor &,
                            const Tensor &, const Tensor &, Tensor &, int64_t, double, int64_t,
                            const OptT &, const OptT &, Tensor &, const OptT &, double,
                            const OptT &) {}
void adam_slabs_meta(Tensor &, Tensor &, Tensor &, Tensor &, const OptT &, const OptT &,
                     const Tensor &, Tensor &, double, double, double, double, double, double,
                     bool) {}
void adam_meta(Tensor &, Tensor &, Tensor &, Tensor &, const OptT &, const OptT &, const Tensor &,
               double, double, double, double, double, bool) {}
void target_sync_meta(const Tensor &, Tensor &, const OptT &, int64_t) {}
void q_argmax_meta(const Tensor &, int64_t, int64_t, const Tensor &, Tensor &, const OptT &, bool) {}

}  // namespace

// The tree digest this operator library was built from (build.py passes it as
// a define; ops.load() compares it with the tree, like libdmdqn_hip.so's).
extern "C" const char *dmdqn_torch_source_digest(void) { return DMDQN_SOURCE_DIGEST; }

// Schemas: each op cites the reference call it replaces (include/dmdqn.h has
// the argument meanings).
TORCH_LIBRARY(dmdqn, m) {
    // random.seed / np.random.seed of the per-replica streams (dqn_agent.py:63, :263-265)
    m.def("mt_seed(Tensor(a!) state, Tensor seeds, str kind) -> ()");
    m.def("mt_draw_u32(Tensor(a!) state, int count, Tensor(b!) out) -> ()");
    // DQNAgent.select_action (dqn_agent.py:246-274)
    // (uniform: test.py:92-93's randint-only draw)
    m.def("act(Tensor(a!) np_state, int A, float eps, int n_actions, Tensor? greedy, "
          "Tensor(b!) actions, bool uniform=False) -> ()");
    // get_own_state / build_state_vector / rewards (order_lanes.py:430-555, train.py:159-165,254)
    m.def("observe(int R, int C, Tensor halt, Tensor phase, Tensor tspent, int mode, "
          "Tensor(a!)? local, Tensor(b!)? obs, Tensor? prev_local, Tensor(c!)? reward) -> ()");
    // ReplayBuffer.add (dqn_agent.py:31-57)
    m.def("replay_store(int slot, Tensor obs_s, Tensor obs_n, Tensor act, Tensor rew, Tensor done, "
          "Tensor(a!) ring_s, Tensor(b!) ring_n, Tensor(c!) ring_a, Tensor(d!) ring_r, "
          "Tensor(e!) ring_d, Tensor(f!) err) -> ()");
    // random.sample(self.buffer, k) (dqn_agent.py:63)
    m.def("replay_sample(Tensor(a!) py_state, int A, int n, int k, Tensor(b!) idx, "
          "int lds_budget=0) -> ()");
    // ReplayBuffer.add / .sample on float rows (the per-agent drop-in, dqn_agent.py:39-64)
    m.def("replay_store_f32(int slot, Tensor obs_s, Tensor obs_n, Tensor act, Tensor rew, "
          "Tensor done, Tensor(a!) rows_s, Tensor(b!) rows_n, Tensor(c!) ring_a, Tensor(d!) ring_r, "
          "Tensor(e!) ring_d) -> ()");
    m.def("replay_gather_f32(Tensor rows_s, Tensor rows_n, Tensor idx, int start, Tensor(a!) xs, "
          "Tensor(b!) xn) -> ()");
    // traci.load (train.py:190); setPhase x A + simulationStep x K (train.py:225-236)
    m.def("sim_reset(Tensor(a!)[] state, Tensor[] tables, int[] dims, Tensor? mask=None) -> ()");
    m.def("sim_step(Tensor(a!)[] state, Tensor[] tables, int[] dims, float[] idm, Tensor? actions, "
          "int stride, int t0, int K, int max_time, Tensor(b!) halt, Tensor(c!) phase, "
          "Tensor(d!) tspent, Tensor(e!) done) -> ()");
    // the env side of one loop iteration in one launch: select_action, setPhase + K
    // substeps, observation / reward, ReplayBuffer.add (train.py:211-282)
    m.def("env_step(Tensor(a!)[] state, Tensor[] tables, int[] dims, float[] idm, int stride, "
          "int t0, int K, int max_time, Tensor(b!) halt, Tensor(c!) phase, Tensor(d!) tspent, "
          "Tensor(e!) done, Tensor(f!) np_state, Tensor? greedy, Tensor(g!) actions, float eps, "
          "int n_actions, int mode, Tensor(h!) local, Tensor(i!) obs, Tensor prev_local, "
          "Tensor(j!) reward, Tensor obs_s, int slot, Tensor(k!) ring_s, Tensor(l!) ring_n, "
          "Tensor(m!) ring_a, Tensor(n!) ring_r, Tensor(o!) ring_d, Tensor(p!) err) -> ()");
    // DQNAgent.learn + the target sync (dqn_agent.py:328-387)
    m.def("learn_step(Tensor ring_s, Tensor ring_n, Tensor ring_a, Tensor ring_d, Tensor ring_r, "
          "Tensor idx, Tensor(a!) params, Tensor(b!) adam_m, Tensor(c!) adam_v, Tensor(d!) target, "
          "Tensor(e!)? target_h, Tensor(f!) loss, int start, int hidden, int precision, bool sync, "
          "float gamma, float alpha, float c1, float c2, float eps, int loss_kind, "
          "Tensor(g!)? qstats, Tensor(h!)? rn_out, Tensor(i!)? stamps, Tensor(j!)? grad=None, "
          "Tensor? xs=None, Tensor? xn=None) -> ()");
    // C5: per-agent gradients of one shared net, summed
    m.def("learn_shared_grad(Tensor ring_s, Tensor ring_n, Tensor ring_a, Tensor ring_d, "
          "Tensor ring_r, Tensor idx, Tensor params, Tensor target, Tensor target_h, "
          "Tensor params_h, Tensor(a!) loss, int start, float gamma, int loss_kind, "
          "Tensor(b!)? qstats, Tensor(c!)? rn_out, Tensor(d!) slab, Tensor(e!)? grad, "
          "float scale, Tensor(f!)? work=None) -> ()");
    // C5, one rank: the slab reduction and the Keras-3 Adam step in one launch
    m.def("adam_slabs(Tensor(a!) params, Tensor(b!) adam_m, Tensor(c!) adam_v, Tensor(d!) target, "
          "Tensor(e!)? target_h, Tensor(f!)? params_h, Tensor slab, Tensor(g!) grad, float scale, "
          "float gscale, float alpha, float c1, float c2, float eps, bool sync) -> ()");
    // Keras-3 Adam (dqn_agent.py:357, A-11) on a flat gradient
    m.def("adam(Tensor(a!) params, Tensor(b!) adam_m, Tensor(c!) adam_v, Tensor(d!) target, "
          "Tensor(e!)? target_h, Tensor(f!)? params_h, Tensor grad, float gscale, float alpha, "
          "float c1, float c2, float eps, bool sync) -> ()");
    // DQNAgent.update_target_network (dqn_agent.py:382-387)
    m.def("target_sync(Tensor params, Tensor(a!) target, Tensor(b!)? target_h, int precision) -> ()");
    // the greedy branch of select_action (dqn_agent.py:268-273)
    m.def("q_argmax(Tensor params, int hidden, int precision, Tensor obs, Tensor(a!) out, "
          "Tensor(b!)? q, bool shared) -> ()");
}

TORCH_LIBRARY_IMPL(dmdqn, CUDA, m) {
    m.impl("mt_seed", &mt_seed);
    m.impl("mt_draw_u32", &mt_draw_u32);
    m.impl("act", &act);
    m.impl("observe", &observe);
    m.impl("replay_store", &replay_store);
    m.impl("replay_sample", &replay_sample);
    m.impl("replay_store_f32", &replay_store_f32);
    m.impl("replay_gather_f32", &replay_gather_f32);
    m.impl("sim_reset", &sim_reset);
    m.impl("sim_step", &sim_step);
    m.impl("env_step", &env_step);
    m.impl("learn_step", &learn_step);
    m.impl("learn_shared_grad", &learn_shared_grad);
    m.impl("adam", &adam);
    m.impl("adam_slabs", &adam_slabs);
    m.impl("target_sync", &target_sync);
    m.impl("q_argmax", &q_argmax);
}

TORCH_LIBRARY_IMPL(dmdqn, Meta, m) {
    m.impl("mt_seed", &mt_seed_meta);
    m.impl("mt_draw_u32", &mt_draw_u32_meta);
    m.impl("act", &act_meta);
    m.impl("observe", &observe_meta);
    m.impl("replay_store", &replay_store_meta);
    m.impl("replay_sample", &replay_sample_meta);
    m.impl("replay_store_f32", &replay_store_f32_meta);
    m.impl("replay_gather_f32", &replay_gather_f32_meta);
    m.impl("sim_reset", &sim_reset_meta);
    m.impl("sim_step", &sim_step_meta);
    m.impl("env_step", &env_step_meta);
    m.impl("learn_step", &learn_step_meta);
    m.impl("learn_shared_grad", &learn_shared_grad_meta);
    m.impl("adam", &adam_meta);
    m.impl("adam_slabs", &adam_slabs_meta);
    m.impl("target_sync", &target_sync_meta);
    m.impl("q_argmax", &q_argmax_meta);
}
