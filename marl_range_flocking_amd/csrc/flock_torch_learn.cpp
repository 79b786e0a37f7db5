// flock_torch_learn.cpp — the learner-side kernels (include/flock_learn.h) as PyTorch custom ops: torch.ops.flock.*
//
// Same conventions as flock_torch.cpp: every buffer an op writes is a mutable alias argument (Tensor(a!)); the ops
// return nothing, enqueue on the current HIP stream of their tensors' device (under a device guard) and never
// synchronise; Meta kernels run the same checks with no launch; errors are TORCH_CHECKs (RuntimeError).
//
//   flock::adam_step         torch.optim.Adam.step() of every agent network at once + the target soft update
//                            (maddpg_official_rnn/agent.py:32-33, net.py:74-78; shared critic
//                            agent_simple_shared_critic.py:141,150,158-185; vdn/train_flock.py:40-43), step count on
//                            the device (graph-capturable)
//   flock::soft_update       the soft update alone (net.py:74-78 mode 0; agent_simple_shared_critic.py:158-185 mode 1)
//   flock::grad_norm         clip_grad_norm_ (vdn/train_flock.py:42) without a host sync
//   flock::gru_cell_fwd/_bwd nn.GRUCell elementwise part (maddpg_official_rnn/net.py:33,118; vdn/net.py:24)
//   flock::gru_seq_fwd/_bwd  a whole chunk of GRUCell steps (vdn/train_flock.py:23-36, MADDPG.py:95-132)
//   flock::gru_seq_q_fwd/_bwd  the same with VDN's q head fused (learners/vdn/net.py:34-37)
//   flock::vdn_feat_fwd/_bwd the VDN QNet feature chain + GRU input side (vdn/net.py:19-33) and its backward
//   flock::gather_rows / scatter_rows / ring_store   replay gather / insert (memory_rnn.py:53-99, vdn/utils.py:18-60,
//                            maddpg_shared_critic/utils.py:47-76)
//   flock::sc_prep_snapshot  shared-critic learn() prologue: Philox row sample + minibatch copy (utils.py:65-76)
//   flock::sc_prep           shared-critic learn() prologue without the snapshot (the agent + Philox row indices)
//   flock::sc_round          shared-critic learn(): critic phase (agent_simple_shared_critic.py:118-141) and / or the
//                            actor phase (:144-155) of two learn() calls in one set of launches
//   flock::sc_round_adam     the Adam half of a data-parallel round (after the gradient all-reduce)
//   flock::sc_act            shared-critic choose_action of every agent on every env row (+ the OU step), one launch
//                            (agent_simple_shared_critic.py:92-107, ddpg_network.py:132-141, utils.py:15-18)
#include <ATen/ATen.h>
#include <ATen/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "flock_learn.h"
#include "flock_torch_sc.h"

namespace {

using at::Tensor;
using c10::optional;

void* stream_of(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }
void rc_check(int rc, const char* fn) { TORCH_CHECK(rc == 0, fn, ": ", flock_learn_last_error()); }
void hip_only(const Tensor& t, const char* op) {
    TORCH_CHECK(t.device().is_cuda(), op, ": flock ops run on a HIP device only (no CPU fallback); got ", t.device());
}

// A tensor traced with symbolic sizes (AOT dispatch with dynamic shapes) has no concrete sizes / numel to compare:
// the Meta kernels skip their shape checks for it (the HIP wrappers always run them on the real tensors).
bool symbolic(const Tensor& t) { return t.defined() && t.unsafeGetTensorImpl()->has_symbolic_sizes_strides(); }
bool sym1(const Tensor& t) { return symbolic(t); }
bool sym1(const optional<Tensor>& t) { return t.has_value() && symbolic(*t); }
bool sym1(at::TensorList l) {
    for (const Tensor& t : l)
        if (symbolic(t)) return true;
    return false;
}
template <typename... Ts>
bool any_sym(const Ts&... ts) { return (sym1(ts) || ...); }

// a dense f32 (or other dtype) buffer on `like`'s device
void dense(const Tensor& t, const char* name, at::ScalarType dtype, const Tensor& like) {
    TORCH_CHECK(t.device() == like.device(), name, " must be on ", like.device(), ", got ", t.device());
    TORCH_CHECK(t.scalar_type() == dtype, name, " must be ", dtype, ", got ", t.scalar_type());
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void shaped(const Tensor& t, const char* name, at::ScalarType dtype, at::IntArrayRef shape, const Tensor& like) {
    dense(t, name, dtype, like);
    TORCH_CHECK(t.sizes() == shape, name, " must have shape ", shape, ", got ", t.sizes());
}
void numel_is(const Tensor& t, const char* name, int64_t n) {
    TORCH_CHECK(t.numel() == n, name, " must have ", n, " elements, got ", t.numel());
}
template <typename T>
T* ptr(const Tensor& t) { return static_cast<T*>(t.data_ptr()); }
template <typename T>
T* ptr(const optional<Tensor>& t) { return t.has_value() ? static_cast<T*>(t->data_ptr()) : nullptr; }

// --------------------------------------------------------------------------------------------------- adam_step
void adam_checks(const Tensor& param, const Tensor& grad, const Tensor& m, const Tensor& v, const Tensor& step,
                 const optional<Tensor>& grad_scale, const optional<Tensor>& target) {
    if (any_sym(param, grad, m, v, step, grad_scale, target)) return;
    const int64_t n = param.numel();
    dense(param, "param", at::kFloat, param);
    dense(grad, "grad", at::kFloat, param);
    dense(m, "exp_avg", at::kFloat, param);
    dense(v, "exp_avg_sq", at::kFloat, param);
    numel_is(grad, "grad", n);
    numel_is(m, "exp_avg", n);
    numel_is(v, "exp_avg_sq", n);
    shaped(step, "step", at::kLong, {1}, param);
    if (grad_scale) {
        dense(*grad_scale, "grad_scale", at::kFloat, param);
        numel_is(*grad_scale, "grad_scale", 1);
    }
    if (target) {
        dense(*target, "target", at::kFloat, param);
        numel_is(*target, "target", n);
    }
}

void adam_step_hip(const Tensor& param, const Tensor& grad, const Tensor& m, const Tensor& v, const Tensor& step,
                   const optional<Tensor>& grad_scale, const optional<Tensor>& target, double lr, double beta1,
                   double beta2, double eps, double tau, int64_t target_mode) {
    hip_only(param, "adam_step");
    adam_checks(param, grad, m, v, step, grad_scale, target);
    TORCH_CHECK(target_mode == 0 || target_mode == 1, "adam_step: target_mode must be 0 or 1");
    const at::OptionalDeviceGuard g(param.device());
    rc_check(flock_adam_step_dev(stream_of(param), param.numel(), ptr<float>(param), ptr<const float>(grad),
                                 ptr<float>(m), ptr<float>(v), ptr<const float>(grad_scale), (float)lr, (float)beta1,
                                 (float)beta2, (float)eps, ptr<const int64_t>(step), ptr<float>(target), (float)tau,
                                 (int)target_mode),
             "flock_adam_step_dev");
}

void adam_step_meta(const Tensor& param, const Tensor& grad, const Tensor& m, const Tensor& v, const Tensor& step,
                    const optional<Tensor>& grad_scale, const optional<Tensor>& target, double, double, double,
                    double, double, int64_t) {
    adam_checks(param, grad, m, v, step, grad_scale, target);
}

// ------------------------------------------------------------------------------------------------- soft_update
void soft_checks(const Tensor& target, const Tensor& src, int64_t mode) {
    if (any_sym(target, src)) return;
    dense(target, "target", at::kFloat, target);
    dense(src, "src", at::kFloat, target);
    numel_is(src, "src", target.numel());
    TORCH_CHECK(mode == 0 || mode == 1, "soft_update: mode must be 0 or 1");
}
void soft_update_hip(const Tensor& target, const Tensor& src, double tau, int64_t mode) {
    hip_only(target, "soft_update");
    soft_checks(target, src, mode);
    const at::OptionalDeviceGuard g(target.device());
    rc_check(flock_soft_update(stream_of(target), target.numel(), ptr<float>(target), ptr<const float>(src),
                               (float)tau, (int)mode),
             "flock_soft_update");
}
void soft_update_meta(const Tensor& target, const Tensor& src, double, int64_t mode) { soft_checks(target, src, mode); }

// --------------------------------------------------------------------------------------------------- grad_norm
void norm_checks(const Tensor& grad, const Tensor& partial, const Tensor& out) {
    if (any_sym(grad, partial, out)) return;
    dense(grad, "grad", at::kFloat, grad);
    dense(partial, "partial", at::kDouble, grad);
    TORCH_CHECK(partial.dim() == 1 && partial.numel() >= 1, "partial must be a 1-D scratch buffer");
    shaped(out, "out", at::kFloat, {2}, grad);
}
void grad_norm_hip(const Tensor& grad, const Tensor& partial, const Tensor& out, double max_norm) {
    hip_only(grad, "grad_norm");
    norm_checks(grad, partial, out);
    const at::OptionalDeviceGuard g(grad.device());
    rc_check(flock_grad_norm(stream_of(grad), grad.numel(), ptr<const float>(grad), ptr<double>(partial),
                             (int)partial.numel(), (float)max_norm, ptr<float>(out)),
             "flock_grad_norm");
}
void grad_norm_meta(const Tensor& grad, const Tensor& partial, const Tensor& out, double) {
    norm_checks(grad, partial, out);
}

// ----------------------------------------------------------------------------------------- gru_cell_fwd / _bwd
// gi, gh [..., 3H]; h, hout [..., H]; ws [..., 4H]
int64_t gru_rows(const Tensor& h) {
    TORCH_CHECK(h.dim() >= 1 && h.size(-1) >= 1, "h must be [..., H]");
    return h.numel() / h.size(-1);
}
void gru_cell_fwd_checks(const Tensor& gi, const Tensor& gh, const Tensor& h, const Tensor& hout,
                         const optional<Tensor>& ws) {
    if (any_sym(gi, gh, h, hout, ws)) return;
    const int64_t rows = gru_rows(h), H = h.size(-1);
    dense(h, "h", at::kFloat, h);
    dense(gi, "gi", at::kFloat, h);
    dense(gh, "gh", at::kFloat, h);
    dense(hout, "hout", at::kFloat, h);
    numel_is(gi, "gi", rows * 3 * H);
    numel_is(gh, "gh", rows * 3 * H);
    numel_is(hout, "hout", rows * H);
    if (ws) {
        dense(*ws, "ws", at::kFloat, h);
        numel_is(*ws, "ws", rows * 4 * H);
    }
}
void gru_cell_fwd_hip(const Tensor& gi, const Tensor& gh, const Tensor& h, const Tensor& hout,
                      const optional<Tensor>& ws) {
    hip_only(h, "gru_cell_fwd");
    gru_cell_fwd_checks(gi, gh, h, hout, ws);
    const at::OptionalDeviceGuard g(h.device());
    rc_check(flock_gru_fwd(stream_of(h), gru_rows(h), (int)h.size(-1), ptr<const float>(gi), ptr<const float>(gh),
                           ptr<const float>(h), ptr<float>(hout), ptr<float>(ws)),
             "flock_gru_fwd");
}
void gru_cell_fwd_meta(const Tensor& gi, const Tensor& gh, const Tensor& h, const Tensor& hout,
                       const optional<Tensor>& ws) {
    gru_cell_fwd_checks(gi, gh, h, hout, ws);
}
void gru_cell_bwd_checks(const Tensor& dhout, const Tensor& h, const Tensor& ws, const Tensor& dgi, const Tensor& dgh,
                         const Tensor& dh) {
    if (any_sym(dhout, h, ws, dgi, dgh, dh)) return;
    const int64_t rows = gru_rows(h), H = h.size(-1);
    dense(h, "h", at::kFloat, h);
    dense(dhout, "dhout", at::kFloat, h);
    dense(ws, "ws", at::kFloat, h);
    dense(dgi, "dgi", at::kFloat, h);
    dense(dgh, "dgh", at::kFloat, h);
    dense(dh, "dh", at::kFloat, h);
    numel_is(dhout, "dhout", rows * H);
    numel_is(ws, "ws", rows * 4 * H);
    numel_is(dgi, "dgi", rows * 3 * H);
    numel_is(dgh, "dgh", rows * 3 * H);
    numel_is(dh, "dh", rows * H);
}
void gru_cell_bwd_hip(const Tensor& dhout, const Tensor& h, const Tensor& ws, const Tensor& dgi, const Tensor& dgh,
                      const Tensor& dh) {
    hip_only(h, "gru_cell_bwd");
    gru_cell_bwd_checks(dhout, h, ws, dgi, dgh, dh);
    const at::OptionalDeviceGuard g(h.device());
    rc_check(flock_gru_bwd(stream_of(h), gru_rows(h), (int)h.size(-1), ptr<const float>(dhout), ptr<const float>(h),
                           ptr<const float>(ws), ptr<float>(dgi), ptr<float>(dgh), ptr<float>(dh)),
             "flock_gru_bwd");
}
void gru_cell_bwd_meta(const Tensor& dhout, const Tensor& h, const Tensor& ws, const Tensor& dgi, const Tensor& dgh,
                       const Tensor& dh) {
    gru_cell_bwd_checks(dhout, h, ws, dgi, dgh, dh);
}

// ------------------------------------------------------------------------------------------ gru_seq_fwd / _bwd
// gi [A, C, B, 3H]; w_hh [A, 3H, H]; b_hh [A, 3H]; keep [C, A, B] bool / uint8, any strides (an expanded view)
void keep_check(const Tensor& keep, int64_t A, int64_t C, int64_t B, const Tensor& like) {
    TORCH_CHECK(keep.device() == like.device(), "keep must be on ", like.device());
    TORCH_CHECK(keep.scalar_type() == at::kBool || keep.scalar_type() == at::kByte, "keep must be bool or uint8");
    TORCH_CHECK(keep.sizes() == at::IntArrayRef({C, A, B}), "keep must be [C, A, B] = [", C, ", ", A, ", ", B,
                "], got ", keep.sizes());
}
void gru_seq_fwd_checks(const Tensor& gi, const Tensor& w_hh, const Tensor& b_hh, const Tensor& keep, const Tensor& hs,
                        const optional<Tensor>& ws) {
    if (any_sym(gi, w_hh, b_hh, keep, hs, ws)) return;
    TORCH_CHECK(gi.dim() == 4 && gi.size(3) % 3 == 0, "gi must be [A, C, B, 3H], got ", gi.sizes());
    const int64_t A = gi.size(0), C = gi.size(1), B = gi.size(2), H = gi.size(3) / 3;
    TORCH_CHECK(H == 32, "gru_seq: hidden size must be 32");
    shaped(gi, "gi", at::kFloat, {A, C, B, 3 * H}, gi);
    shaped(w_hh, "w_hh", at::kFloat, {A, 3 * H, H}, gi);
    shaped(b_hh, "b_hh", at::kFloat, {A, 3 * H}, gi);
    keep_check(keep, A, C, B, gi);
    shaped(hs, "hs", at::kFloat, {A, C, B, H}, gi);
    if (ws) shaped(*ws, "ws", at::kFloat, {A, C, B, 4 * H}, gi);
}
void gru_seq_fwd_hip(const Tensor& gi, const Tensor& w_hh, const Tensor& b_hh, const Tensor& keep, const Tensor& hs,
                     const optional<Tensor>& ws) {
    hip_only(gi, "gru_seq_fwd");
    gru_seq_fwd_checks(gi, w_hh, b_hh, keep, hs, ws);
    const at::OptionalDeviceGuard g(gi.device());
    rc_check(flock_gru_seq_fwd(stream_of(gi), (int)gi.size(0), (int)gi.size(1), (int)gi.size(2), (int)gi.size(3) / 3,
                               ptr<const float>(gi), ptr<const float>(w_hh), ptr<const float>(b_hh),
                               static_cast<const uint8_t*>(keep.data_ptr()), keep.stride(0), keep.stride(1),
                               keep.stride(2), ptr<float>(hs), ptr<float>(ws)),
             "flock_gru_seq_fwd");
}
void gru_seq_fwd_meta(const Tensor& gi, const Tensor& w_hh, const Tensor& b_hh, const Tensor& keep, const Tensor& hs,
                      const optional<Tensor>& ws) {
    gru_seq_fwd_checks(gi, w_hh, b_hh, keep, hs, ws);
}
void gru_seq_bwd_checks(const Tensor& dhs, const Tensor& hs, const Tensor& ws, const Tensor& w_hh, const Tensor& keep,
                        const Tensor& dgi, const Tensor& dw_hh, const Tensor& db_hh) {
    if (any_sym(dhs, hs, ws, w_hh, keep, dgi, dw_hh, db_hh)) return;
    TORCH_CHECK(hs.dim() == 4, "hs must be [A, C, B, H], got ", hs.sizes());
    const int64_t A = hs.size(0), C = hs.size(1), B = hs.size(2), H = hs.size(3);
    TORCH_CHECK(H == 32, "gru_seq: hidden size must be 32");
    shaped(hs, "hs", at::kFloat, {A, C, B, H}, hs);
    shaped(dhs, "dhs", at::kFloat, {A, C, B, H}, hs);
    shaped(ws, "ws", at::kFloat, {A, C, B, 4 * H}, hs);
    shaped(w_hh, "w_hh", at::kFloat, {A, 3 * H, H}, hs);
    keep_check(keep, A, C, B, hs);
    shaped(dgi, "dgi", at::kFloat, {A, C, B, 3 * H}, hs);
    shaped(dw_hh, "dw_hh", at::kFloat, {A, 3 * H, H}, hs);
    shaped(db_hh, "db_hh", at::kFloat, {A, 3 * H}, hs);
}
void gru_seq_bwd_hip(const Tensor& dhs, const Tensor& hs, const Tensor& ws, const Tensor& w_hh, const Tensor& keep,
                     const Tensor& dgi, const Tensor& dw_hh, const Tensor& db_hh) {
    hip_only(hs, "gru_seq_bwd");
    gru_seq_bwd_checks(dhs, hs, ws, w_hh, keep, dgi, dw_hh, db_hh);
    const at::OptionalDeviceGuard g(hs.device());
    rc_check(flock_gru_seq_bwd(stream_of(hs), (int)hs.size(0), (int)hs.size(1), (int)hs.size(2), (int)hs.size(3),
                               ptr<const float>(dhs), ptr<const float>(hs), ptr<const float>(ws),
                               ptr<const float>(w_hh), static_cast<const uint8_t*>(keep.data_ptr()), keep.stride(0),
                               keep.stride(1), keep.stride(2), ptr<float>(dgi), ptr<float>(dw_hh), ptr<float>(db_hh)),
             "flock_gru_seq_bwd");
}
void gru_seq_bwd_meta(const Tensor& dhs, const Tensor& hs, const Tensor& ws, const Tensor& w_hh, const Tensor& keep,
                      const Tensor& dgi, const Tensor& dw_hh, const Tensor& db_hh) {
    gru_seq_bwd_checks(dhs, hs, ws, w_hh, keep, dgi, dw_hh, db_hh);
}

// ---------------------------------------------------------------------------------- gru_seq_q_fwd / gru_seq_q_bwd
// the recurrence with VDN's q head fused: w_q [A, NA, H], b_q [A, NA], q [A, C, B, NA]; hs / ws optional together
void gru_seq_q_fwd_checks(const Tensor& gi, const Tensor& w_hh, const Tensor& b_hh, const Tensor& w_q,
                          const Tensor& b_q, const Tensor& keep, const optional<Tensor>& hs,
                          const optional<Tensor>& ws, const Tensor& q) {
    if (any_sym(gi, w_hh, b_hh, w_q, b_q, keep, hs, ws, q)) return;
    TORCH_CHECK(gi.dim() == 4 && gi.size(3) % 3 == 0, "gi must be [A, C, B, 3H], got ", gi.sizes());
    const int64_t A = gi.size(0), C = gi.size(1), B = gi.size(2), H = gi.size(3) / 3;
    TORCH_CHECK(H == 32, "gru_seq_q: hidden size must be 32");
    TORCH_CHECK(w_q.dim() == 3 && w_q.size(1) >= 1 && w_q.size(1) <= 16, "w_q must be [A, NA <= 16, H]");
    const int64_t NA = w_q.size(1);
    shaped(gi, "gi", at::kFloat, {A, C, B, 3 * H}, gi);
    shaped(w_hh, "w_hh", at::kFloat, {A, 3 * H, H}, gi);
    shaped(b_hh, "b_hh", at::kFloat, {A, 3 * H}, gi);
    shaped(w_q, "w_q", at::kFloat, {A, NA, H}, gi);
    shaped(b_q, "b_q", at::kFloat, {A, NA}, gi);
    keep_check(keep, A, C, B, gi);
    TORCH_CHECK(hs.has_value() == ws.has_value(), "gru_seq_q_fwd: hs and ws are given together (the backward's)");
    if (hs) shaped(*hs, "hs", at::kFloat, {A, C, B, H}, gi);
    if (ws) shaped(*ws, "ws", at::kFloat, {A, C, B, 4 * H}, gi);
    shaped(q, "q", at::kFloat, {A, C, B, NA}, gi);
}
void gru_seq_q_fwd_hip(const Tensor& gi, const Tensor& w_hh, const Tensor& b_hh, const Tensor& w_q, const Tensor& b_q,
                       const Tensor& keep, const optional<Tensor>& hs, const optional<Tensor>& ws, const Tensor& q) {
    hip_only(gi, "gru_seq_q_fwd");
    gru_seq_q_fwd_checks(gi, w_hh, b_hh, w_q, b_q, keep, hs, ws, q);
    const at::OptionalDeviceGuard g(gi.device());
    rc_check(flock_gru_seq_q_fwd(stream_of(gi), (int)gi.size(0), (int)gi.size(1), (int)gi.size(2),
                                 (int)gi.size(3) / 3, (int)w_q.size(1), ptr<const float>(gi), ptr<const float>(w_hh),
                                 ptr<const float>(b_hh), ptr<const float>(w_q), ptr<const float>(b_q),
                                 static_cast<const uint8_t*>(keep.data_ptr()), keep.stride(0), keep.stride(1),
                                 keep.stride(2), ptr<float>(hs), ptr<float>(ws), ptr<float>(q)),
             "flock_gru_seq_q_fwd");
}
void gru_seq_q_fwd_meta(const Tensor& gi, const Tensor& w_hh, const Tensor& b_hh, const Tensor& w_q,
                        const Tensor& b_q, const Tensor& keep, const optional<Tensor>& hs, const optional<Tensor>& ws,
                        const Tensor& q) {
    gru_seq_q_fwd_checks(gi, w_hh, b_hh, w_q, b_q, keep, hs, ws, q);
}
void gru_seq_q_bwd_checks(const Tensor& dq, const Tensor& hs, const Tensor& ws, const Tensor& w_hh, const Tensor& w_q,
                          const Tensor& keep, const Tensor& dgi, const Tensor& dw_hh, const Tensor& db_hh,
                          const Tensor& dw_q, const Tensor& db_q) {
    if (any_sym(dq, hs, ws, w_hh, w_q, keep, dgi, dw_hh, db_hh, dw_q, db_q)) return;
    TORCH_CHECK(hs.dim() == 4, "hs must be [A, C, B, H], got ", hs.sizes());
    const int64_t A = hs.size(0), C = hs.size(1), B = hs.size(2), H = hs.size(3);
    TORCH_CHECK(H == 32, "gru_seq_q: hidden size must be 32");
    TORCH_CHECK(w_q.dim() == 3 && w_q.size(1) >= 1 && w_q.size(1) <= 16, "w_q must be [A, NA <= 16, H]");
    const int64_t NA = w_q.size(1);
    shaped(hs, "hs", at::kFloat, {A, C, B, H}, hs);
    shaped(dq, "dq", at::kFloat, {A, C, B, NA}, hs);
    shaped(ws, "ws", at::kFloat, {A, C, B, 4 * H}, hs);
    shaped(w_hh, "w_hh", at::kFloat, {A, 3 * H, H}, hs);
    shaped(w_q, "w_q", at::kFloat, {A, NA, H}, hs);
    keep_check(keep, A, C, B, hs);
    shaped(dgi, "dgi", at::kFloat, {A, C, B, 3 * H}, hs);
    shaped(dw_hh, "dw_hh", at::kFloat, {A, 3 * H, H}, hs);
    shaped(db_hh, "db_hh", at::kFloat, {A, 3 * H}, hs);
    shaped(dw_q, "dw_q", at::kFloat, {A, NA, H}, hs);
    shaped(db_q, "db_q", at::kFloat, {A, NA}, hs);
}
void gru_seq_q_bwd_hip(const Tensor& dq, const Tensor& hs, const Tensor& ws, const Tensor& w_hh, const Tensor& w_q,
                       const Tensor& keep, const Tensor& dgi, const Tensor& dw_hh, const Tensor& db_hh,
                       const Tensor& dw_q, const Tensor& db_q) {
    hip_only(hs, "gru_seq_q_bwd");
    gru_seq_q_bwd_checks(dq, hs, ws, w_hh, w_q, keep, dgi, dw_hh, db_hh, dw_q, db_q);
    const at::OptionalDeviceGuard g(hs.device());
    rc_check(flock_gru_seq_q_bwd(stream_of(hs), (int)hs.size(0), (int)hs.size(1), (int)hs.size(2), (int)hs.size(3),
                                 (int)w_q.size(1), ptr<const float>(dq), ptr<const float>(hs), ptr<const float>(ws),
                                 ptr<const float>(w_hh), ptr<const float>(w_q),
                                 static_cast<const uint8_t*>(keep.data_ptr()), keep.stride(0), keep.stride(1),
                                 keep.stride(2), ptr<float>(dgi), ptr<float>(dw_hh), ptr<float>(db_hh),
                                 ptr<float>(dw_q), ptr<float>(db_q)),
             "flock_gru_seq_q_bwd");
}
void gru_seq_q_bwd_meta(const Tensor& dq, const Tensor& hs, const Tensor& ws, const Tensor& w_hh, const Tensor& w_q,
                        const Tensor& keep, const Tensor& dgi, const Tensor& dw_hh, const Tensor& db_hh,
                        const Tensor& dw_q, const Tensor& db_q) {
    gru_seq_q_bwd_checks(dq, hs, ws, w_hh, w_q, keep, dgi, dw_hh, db_hh, dw_q, db_q);
}

// ------------------------------------------------------------------------------------------------ vdn_feat_fwd
// x [A, C, B, n] (any strides with a unit feature stride); w1 [A,64,n] b1 [A,64] w2 [A,32,64] b2 [A,32] w_ih [A,96,32]
// b_ih [A,96]; y1 [A, C*B, 64], y2 [A, C*B, 32] (optional), gi [A, C*B, 96]
void vdn_feat_checks(const Tensor& x, const Tensor& w1, const Tensor& b1, const Tensor& w2, const Tensor& b2,
                     const Tensor& wi, const Tensor& bi, const optional<Tensor>& y1, const optional<Tensor>& y2,
                     const Tensor& gi) {
    if (any_sym(x, w1, b1, w2, b2, wi, bi, y1, y2, gi)) return;
    TORCH_CHECK(x.dim() == 4, "x must be [A, C, B, n_obs], got ", x.sizes());
    const int64_t A = x.size(0), R = x.size(1) * x.size(2), n = x.size(3);
    TORCH_CHECK(n >= 1 && n <= 16, "vdn_feat_fwd: n_obs must be in [1, 16]");
    TORCH_CHECK(x.scalar_type() == at::kFloat && x.stride(3) == 1, "x must be f32 with a unit feature stride");
    shaped(w1, "w1", at::kFloat, {A, 64, n}, x);
    shaped(b1, "b1", at::kFloat, {A, 64}, x);
    shaped(w2, "w2", at::kFloat, {A, 32, 64}, x);
    shaped(b2, "b2", at::kFloat, {A, 32}, x);
    shaped(wi, "w_ih", at::kFloat, {A, 96, 32}, x);
    shaped(bi, "b_ih", at::kFloat, {A, 96}, x);
    if (y1) shaped(*y1, "y1", at::kFloat, {A, R, 64}, x);
    if (y2) shaped(*y2, "y2", at::kFloat, {A, R, 32}, x);
    shaped(gi, "gi", at::kFloat, {A, R, 96}, x);
}
void vdn_feat_fwd_hip(const Tensor& x, const Tensor& w1, const Tensor& b1, const Tensor& w2, const Tensor& b2,
                      const Tensor& wi, const Tensor& bi, const optional<Tensor>& y1, const optional<Tensor>& y2,
                      const Tensor& gi) {
    hip_only(x, "vdn_feat_fwd");
    vdn_feat_checks(x, w1, b1, w2, b2, wi, bi, y1, y2, gi);
    const at::OptionalDeviceGuard g(x.device());
    rc_check(flock_vdn_feat_fwd(stream_of(x), (int)x.size(0), (int)(x.size(1) * x.size(2)), (int)x.size(2),
                                (int)x.size(3), ptr<const float>(x), x.stride(0), x.stride(1), x.stride(2),
                                ptr<const float>(w1), ptr<const float>(b1), ptr<const float>(w2),
                                ptr<const float>(b2), ptr<const float>(wi), ptr<const float>(bi), ptr<float>(y1),
                                ptr<float>(y2), ptr<float>(gi)),
             "flock_vdn_feat_fwd");
}
void vdn_feat_fwd_meta(const Tensor& x, const Tensor& w1, const Tensor& b1, const Tensor& w2, const Tensor& b2,
                       const Tensor& wi, const Tensor& bi, const optional<Tensor>& y1, const optional<Tensor>& y2,
                       const Tensor& gi) {
    vdn_feat_checks(x, w1, b1, w2, b2, wi, bi, y1, y2, gi);
}

// backward of the chain (flock_vdn_feat_bwd): dgi [A, C*B, 96], y1 / y2 the forward's outputs -> dw1 [A,64,n],
// db1 [A,64], dw2 [A,32,64], db2 [A,32], dw_ih [A,96,32], db_ih [A,96]
void vdn_feat_bwd_checks(const Tensor& x, const Tensor& w2, const Tensor& wi, const Tensor& y1, const Tensor& y2,
                         const Tensor& dgi, const Tensor& dw1, const Tensor& db1, const Tensor& dw2, const Tensor& db2,
                         const Tensor& dwi, const Tensor& dbi) {
    if (any_sym(x, w2, wi, y1, y2, dgi, dw1, db1, dw2, db2, dwi, dbi)) return;
    TORCH_CHECK(x.dim() == 4, "x must be [A, C, B, n_obs], got ", x.sizes());
    const int64_t A = x.size(0), R = x.size(1) * x.size(2), n = x.size(3);
    TORCH_CHECK(n >= 1 && n <= 16, "vdn_feat_bwd: n_obs must be in [1, 16]");
    TORCH_CHECK(x.scalar_type() == at::kFloat && x.stride(3) == 1, "x must be f32 with a unit feature stride");
    shaped(w2, "w2", at::kFloat, {A, 32, 64}, x);
    shaped(wi, "w_ih", at::kFloat, {A, 96, 32}, x);
    shaped(y1, "y1", at::kFloat, {A, R, 64}, x);
    shaped(y2, "y2", at::kFloat, {A, R, 32}, x);
    shaped(dgi, "dgi", at::kFloat, {A, R, 96}, x);
    shaped(dw1, "dw1", at::kFloat, {A, 64, n}, x);
    shaped(db1, "db1", at::kFloat, {A, 64}, x);
    shaped(dw2, "dw2", at::kFloat, {A, 32, 64}, x);
    shaped(db2, "db2", at::kFloat, {A, 32}, x);
    shaped(dwi, "dw_ih", at::kFloat, {A, 96, 32}, x);
    shaped(dbi, "db_ih", at::kFloat, {A, 96}, x);
}
void vdn_feat_bwd_hip(const Tensor& x, const Tensor& w2, const Tensor& wi, const Tensor& y1, const Tensor& y2,
                      const Tensor& dgi, const Tensor& dw1, const Tensor& db1, const Tensor& dw2, const Tensor& db2,
                      const Tensor& dwi, const Tensor& dbi) {
    hip_only(x, "vdn_feat_bwd");
    vdn_feat_bwd_checks(x, w2, wi, y1, y2, dgi, dw1, db1, dw2, db2, dwi, dbi);
    const at::OptionalDeviceGuard g(x.device());
    rc_check(flock_vdn_feat_bwd(stream_of(x), (int)x.size(0), (int)(x.size(1) * x.size(2)), (int)x.size(2),
                                (int)x.size(3), ptr<const float>(x), x.stride(0), x.stride(1), x.stride(2),
                                ptr<const float>(w2), ptr<const float>(wi), ptr<const float>(y1), ptr<const float>(y2),
                                ptr<const float>(dgi), ptr<float>(dw1), ptr<float>(db1), ptr<float>(dw2),
                                ptr<float>(db2), ptr<float>(dwi), ptr<float>(dbi)),
             "flock_vdn_feat_bwd");
}
void vdn_feat_bwd_meta(const Tensor& x, const Tensor& w2, const Tensor& wi, const Tensor& y1, const Tensor& y2,
                       const Tensor& dgi, const Tensor& dw1, const Tensor& db1, const Tensor& dw2, const Tensor& db2,
                       const Tensor& dwi, const Tensor& dbi) {
    vdn_feat_bwd_checks(x, w2, wi, y1, y2, dgi, dw1, db1, dw2, db2, dwi, dbi);
}

// --------------------------------------------------------------------------------- gather_rows / scatter_rows
// src / dst: [rows_src, ...] f32 rows of `width` floats; idx: int64 of any shape; gather: dst [idx.numel(), width],
// scatter: src [idx.numel(), width]
void rows_checks(const Tensor& src, const Tensor& idx, const Tensor& dst, bool scatter) {
    if (any_sym(src, idx, dst)) return;
    dense(src, "src", at::kFloat, src);
    dense(dst, "dst", at::kFloat, src);
    dense(idx, "idx", at::kLong, src);
    const Tensor& table = scatter ? dst : src;
    const Tensor& rows = scatter ? src : dst;
    TORCH_CHECK(table.dim() >= 1 && table.size(0) >= 1, scatter ? "dst" : "src", " must be [rows, ...]");
    const int64_t width = table.numel() / table.size(0);
    numel_is(rows, scatter ? "src" : "dst", idx.numel() * width);
}
void gather_rows_hip(const Tensor& src, const Tensor& idx, const Tensor& dst) {
    hip_only(src, "gather_rows");
    rows_checks(src, idx, dst, false);
    const at::OptionalDeviceGuard g(src.device());
    rc_check(flock_gather_rows(stream_of(src), idx.numel(), src.numel() / src.size(0), ptr<const float>(src),
                               ptr<const int64_t>(idx), ptr<float>(dst)),
             "flock_gather_rows");
}
void gather_rows_meta(const Tensor& src, const Tensor& idx, const Tensor& dst) { rows_checks(src, idx, dst, false); }
void scatter_rows_hip(const Tensor& src, const Tensor& idx, const Tensor& dst) {
    hip_only(src, "scatter_rows");
    rows_checks(src, idx, dst, true);
    const at::OptionalDeviceGuard g(src.device());
    rc_check(flock_scatter_rows(stream_of(src), idx.numel(), dst.numel() / dst.size(0), ptr<const float>(src),
                                ptr<const int64_t>(idx), ptr<float>(dst)),
             "flock_scatter_rows");
}
void scatter_rows_meta(const Tensor& src, const Tensor& idx, const Tensor& dst) { rows_checks(src, idx, dst, true); }

// -------------------------------------------------------------------------------------------------- ring_store
// src[i]: n rows of field i (f32 [n, w]; kind 1/2 u8|bool [n, w]; kind 3 int64 [n, w]); dst[i]: [capacity, w] f32
void ring_checks(at::TensorList src, at::TensorList dst, at::IntArrayRef kind, int64_t start) {
    if (dst.empty() || any_sym(src, dst)) return;
    TORCH_CHECK(src.size() >= 1 && src.size() <= 8 && dst.size() == src.size() && kind.size() == src.size(),
                "ring_store: 1..8 fields with one dst and one kind each");
    const Tensor& like = dst[0];
    TORCH_CHECK(like.dim() >= 1, "ring_store: dst must be [capacity, ...]");
    const int64_t cap = like.size(0), n = src[0].dim() ? src[0].size(0) : 0;
    TORCH_CHECK(n <= cap && start >= 0 && start < cap, "ring_store: need n <= capacity and 0 <= start < capacity");
    for (size_t i = 0; i < src.size(); ++i) {
        dense(dst[i], "dst", at::kFloat, like);
        TORCH_CHECK(dst[i].size(0) == cap, "ring_store: every dst needs the same capacity");
        TORCH_CHECK(kind[i] >= 0 && kind[i] <= 3, "ring_store: kind must be 0..3");
        const at::ScalarType want = kind[i] == 0 ? at::kFloat : kind[i] == 3 ? at::kLong : src[i].scalar_type();
        TORCH_CHECK(kind[i] == 0 || kind[i] == 3 || want == at::kBool || want == at::kByte,
                    "ring_store: kind 1 / 2 take bool or uint8 rows");
        dense(src[i], "src", want, like);
        const int64_t w = dst[i].numel() / cap;
        numel_is(src[i], "src", n * w);
    }
}
void ring_store_hip(at::TensorList src, at::TensorList dst, at::IntArrayRef kind, int64_t start) {
    hip_only(dst[0], "ring_store");
    ring_checks(src, dst, kind, start);
    const at::OptionalDeviceGuard g(dst[0].device());
    FlockRingField f[8];
    const int64_t cap = dst[0].size(0);
    for (size_t i = 0; i < src.size(); ++i)
        f[i] = FlockRingField{src[i].data_ptr(), ptr<float>(dst[i]), dst[i].numel() / cap, (int)kind[i]};
    rc_check(flock_ring_store(stream_of(dst[0]), src[0].size(0), cap, start, (int)src.size(), f), "flock_ring_store");
}
void ring_store_meta(at::TensorList src, at::TensorList dst, at::IntArrayRef kind, int64_t start) {
    ring_checks(src, dst, kind, start);
}

// -------------------------------------------------------------------------------------- shared critic (flock_sc)
// rows: [state [R, in], new_state [R, in], action [R, na], reward [R] | [R, 1], terminal [R]]
FlockScRows sc_rows(at::TensorList t) {
    return FlockScRows{ptr<float>(t[0]), ptr<float>(t[1]), ptr<float>(t[2]), ptr<float>(t[3]), ptr<float>(t[4])};
}
void sc_rows_check(at::TensorList t, const char* what, int64_t in_dim, int64_t na, const Tensor& like) {
    TORCH_CHECK(t.size() == 5, what, ": [state, new_state, action, reward, terminal]");
    const int64_t R = t[0].dim() ? t[0].size(0) : 0;
    TORCH_CHECK(R >= 1, what, ": empty rows");
    const int64_t w[5] = {in_dim, in_dim, na, 1, 1};
    const char* names[5] = {"state", "new_state", "action", "reward", "terminal"};
    for (int i = 0; i < 5; ++i) {
        dense(t[i], names[i], at::kFloat, like);
        TORCH_CHECK(t[i].dim() >= 1 && t[i].size(0) == R, what, ": every field needs ", R, " rows");
        numel_is(t[i], names[i], R * w[i]);
    }
}
void snapshot_checks(at::TensorList ring, at::TensorList staging, const Tensor& agent_out,
                     const optional<Tensor>& idx_out, int64_t rows) {
    if (ring.empty() || any_sym(ring, staging, agent_out, idx_out)) return;
    TORCH_CHECK(ring.size() == 5 && staging.size() == 5, "sc_prep_snapshot: 5 ring and 5 staging fields");
    const int64_t in_dim = ring[0].dim() == 2 ? ring[0].size(1) : 0;
    const int64_t na = ring[2].dim() == 2 ? ring[2].size(1) : 0;
    TORCH_CHECK(in_dim >= 1 && na >= 1, "sc_prep_snapshot: ring state / action must be [R, in] / [R, na]");
    sc_rows_check(ring, "ring", in_dim, na, ring[0]);
    sc_rows_check(staging, "staging", in_dim, na, ring[0]);
    TORCH_CHECK(rows >= 1 && rows <= ring[0].size(0), "sc_prep_snapshot: 1 <= rows <= ring capacity");
    shaped(agent_out, "agent_out", at::kLong, {1}, ring[0]);
    if (idx_out) shaped(*idx_out, "idx_out", at::kLong, {staging[0].size(0)}, ring[0]);
}
void sc_prep_snapshot_hip(at::TensorList ring, at::TensorList staging, const Tensor& agent_out,
                          const optional<Tensor>& idx_out, int64_t rows, int64_t seed, int64_t counter,
                          int64_t agent) {
    hip_only(agent_out, "sc_prep_snapshot");
    snapshot_checks(ring, staging, agent_out, idx_out, rows);
    const at::OptionalDeviceGuard g(agent_out.device());
    const FlockScRows r = sc_rows(ring), s = sc_rows(staging);
    rc_check(flock_sc_prep_snapshot(stream_of(agent_out), (int)staging[0].size(0), rows, (uint64_t)seed,
                                    (uint64_t)counter, ptr<int64_t>(idx_out), ptr<int64_t>(agent_out), agent,
                                    (int)ring[0].size(1), (int)ring[2].size(1), &r, &s),
             "flock_sc_prep_snapshot");
}
void sc_prep_snapshot_meta(at::TensorList ring, at::TensorList staging, const Tensor& agent_out,
                           const optional<Tensor>& idx_out, int64_t rows, int64_t, int64_t, int64_t) {
    snapshot_checks(ring, staging, agent_out, idx_out, rows);
}

// learner = [critic, critic_grad, critic_exp_avg, critic_exp_avg_sq, critic_step [1] i64, actors, actors_grad,
//            actors_exp_avg, actors_exp_avg_sq, actors_target, actor_steps [n_agents] i64, losses [2],
//            counters [2] i32]
// job     = [] (no phase) or [idx [B] i64, agent [1] i64, state, new_state, action, reward, terminal (the rows the
//            update reads: a staging slot or the ring), workspace, critic_view (empty: none)(, actor_grad_out)]
// dims    = [B, in_dim, n_actions, fc1, fc2, update_rate, do_adam]; hyper = [alpha, beta, gamma, beta1, beta2, eps, tau]
}  // namespace

namespace flock_torch {

void sc_round_checks(at::TensorList L, at::TensorList job, at::IntArrayRef dims, at::ArrayRef<double> hyper,
                     const char* what) {
    if (L.empty() || any_sym(L, job)) return;
    TORCH_CHECK(L.size() == 13, "sc_round: learner must hold the 13 state tensors");
    TORCH_CHECK(dims.size() == 7 && hyper.size() == 7, "sc_round: dims [7] and hyper [7]");
    const Tensor& like = L[0];
    const char* names[13] = {"critic", "critic_grad", "critic_exp_avg", "critic_exp_avg_sq", "critic_step",
                             "actors", "actors_grad", "actors_exp_avg", "actors_exp_avg_sq", "actors_target",
                             "actor_steps", "losses", "counters"};
    for (int i = 0; i < 13; ++i)
        dense(L[i], names[i], i == 4 || i == 10 ? at::kLong : i == 12 ? at::kInt : at::kFloat, like);
    numel_is(L[1], "critic_grad", L[0].numel());
    numel_is(L[2], "critic_exp_avg", L[0].numel());
    numel_is(L[3], "critic_exp_avg_sq", L[0].numel());
    numel_is(L[4], "critic_step", 1);
    for (int i = 6; i <= 9; ++i) numel_is(L[i], names[i], L[5].numel());
    TORCH_CHECK(L[10].numel() >= 1 && L[5].numel() % L[10].numel() == 0, "actor_steps: one per agent");
    numel_is(L[11], "losses", 2);
    numel_is(L[12], "counters", 2);
    if (job.empty()) return;
    TORCH_CHECK(job.size() == 9 || job.size() == 10, what, ": [idx, agent, state, new_state, action, reward, "
                "terminal, workspace, critic_view(, actor_grad_out)]");
    shaped(job[0], "idx", at::kLong, {dims[0]}, like);
    shaped(job[1], "agent", at::kLong, {1}, like);
    sc_rows_check(job.slice(2, 5), what, dims[1], dims[2], like);
    dense(job[7], "workspace", at::kFloat, like);
    numel_is(job[7], "workspace", flock_sc_workspace_floats((int)dims[0], (int)dims[1], (int)dims[2], (int)dims[3],
                                                            (int)dims[4]));
    if (job[8].numel() > 0) {  // an empty critic_view: none (FlockScUpdate.critic_view = NULL)
        dense(job[8], "critic_view", at::kFloat, like);
        numel_is(job[8], "critic_view", L[0].numel());
    }
    if (job.size() == 10) {  // FlockScUpdate.actor_grad_out: one actor's gradient (data-parallel bucket)
        dense(job[9], "actor_grad_out", at::kFloat, like);
        numel_is(job[9], "actor_grad_out", L[5].numel() / L[10].numel());
    }
}
FlockScUpdate sc_update(at::TensorList L, at::TensorList job, at::IntArrayRef dims, at::ArrayRef<double> hyper) {
    FlockScUpdate u{};
    u.B = (int)dims[0];
    u.in_dim = (int)dims[1];
    u.n_actions = (int)dims[2];
    u.fc1 = (int)dims[3];
    u.fc2 = (int)dims[4];
    u.update_rate = (int)dims[5];
    u.do_adam = (int)dims[6];
    u.idx = ptr<const int64_t>(job[0]);
    u.agent = ptr<const int64_t>(job[1]);
    u.ring_state = ptr<const float>(job[2]);
    u.ring_new_state = ptr<const float>(job[3]);
    u.ring_action = ptr<const float>(job[4]);
    u.ring_reward = ptr<const float>(job[5]);
    u.ring_terminal = ptr<const float>(job[6]);
    u.critic = ptr<float>(L[0]);
    u.critic_grad = ptr<float>(L[1]);
    u.critic_exp_avg = ptr<float>(L[2]);
    u.critic_exp_avg_sq = ptr<float>(L[3]);
    u.critic_step = ptr<int64_t>(L[4]);
    u.actors = ptr<float>(L[5]);
    u.actors_grad = ptr<float>(L[6]);
    u.actors_exp_avg = ptr<float>(L[7]);
    u.actors_exp_avg_sq = ptr<float>(L[8]);
    u.actors_target = ptr<float>(L[9]);
    u.actor_steps = ptr<int64_t>(L[10]);
    u.actor_stride = L[5].numel() / L[10].numel();
    u.losses = ptr<float>(L[11]);
    u.workspace = ptr<float>(job[7]);
    u.counters = static_cast<unsigned*>(L[12].data_ptr());
    u.alpha = (float)hyper[0];
    u.beta = (float)hyper[1];
    u.gamma = (float)hyper[2];
    u.beta1 = (float)hyper[3];
    u.beta2 = (float)hyper[4];
    u.eps = (float)hyper[5];
    u.tau = (float)hyper[6];
    u.critic_view = job[8].numel() > 0 ? ptr<float>(job[8]) : nullptr;
    u.actor_grad_out = job.size() == 10 ? ptr<float>(job[9]) : nullptr;
    return u;
}
}  // namespace flock_torch

namespace {

using flock_torch::sc_round_checks;
using flock_torch::sc_update;

void sc_round_hip(at::TensorList learner, at::TensorList critic_job, at::TensorList actor_job, at::IntArrayRef dims,
                  at::ArrayRef<double> hyper) {
    TORCH_CHECK(!learner.empty(), "sc_round: empty learner state");
    hip_only(learner[0], "sc_round");
    TORCH_CHECK(!critic_job.empty() || !actor_job.empty(), "sc_round: neither a critic nor an actor phase");
    sc_round_checks(learner, critic_job, dims, hyper, "critic_job");
    sc_round_checks(learner, actor_job, dims, hyper, "actor_job");
    const at::OptionalDeviceGuard g(learner[0].device());
    FlockScUpdate uc{}, ua{};
    if (!critic_job.empty()) uc = sc_update(learner, critic_job, dims, hyper);
    if (!actor_job.empty()) ua = sc_update(learner, actor_job, dims, hyper);
    rc_check(flock_sc_round(stream_of(learner[0]), critic_job.empty() ? nullptr : &uc,
                            actor_job.empty() ? nullptr : &ua),
             "flock_sc_round");
}
void sc_round_meta(at::TensorList learner, at::TensorList critic_job, at::TensorList actor_job, at::IntArrayRef dims,
                   at::ArrayRef<double> hyper) {
    TORCH_CHECK(!learner.empty(), "sc_round: empty learner state");
    TORCH_CHECK(!critic_job.empty() || !actor_job.empty(), "sc_round: neither a critic nor an actor phase");
    sc_round_checks(learner, critic_job, dims, hyper, "critic_job");
    sc_round_checks(learner, actor_job, dims, hyper, "actor_job");
}

// the Adam half of a data-parallel round (flock_sc_round_adam): after sc_round with do_adam = 0 and the caller's
// all-reduce (sums), Adam on the critic and / or the actor of actor_job's agent, gradients scaled by *grad_scale
void sc_round_adam_hip(at::TensorList learner, at::TensorList critic_job, at::TensorList actor_job,
                       at::IntArrayRef dims, at::ArrayRef<double> hyper, const optional<Tensor>& grad_scale) {
    TORCH_CHECK(!learner.empty(), "sc_round_adam: empty learner state");
    hip_only(learner[0], "sc_round_adam");
    TORCH_CHECK(!critic_job.empty() || !actor_job.empty(), "sc_round_adam: neither a critic nor an actor phase");
    TORCH_CHECK(dims.size() == 7 && dims[6] == 1, "sc_round_adam: dims[6] (do_adam) must be 1");
    sc_round_checks(learner, critic_job, dims, hyper, "critic_job");
    sc_round_checks(learner, actor_job, dims, hyper, "actor_job");
    if (grad_scale) shaped(*grad_scale, "grad_scale", at::kFloat, {1}, learner[0]);
    const at::OptionalDeviceGuard g(learner[0].device());
    FlockScUpdate uc{}, ua{};
    if (!critic_job.empty()) uc = sc_update(learner, critic_job, dims, hyper);
    if (!actor_job.empty()) ua = sc_update(learner, actor_job, dims, hyper);
    rc_check(flock_sc_round_adam(stream_of(learner[0]), critic_job.empty() ? nullptr : &uc,
                                 actor_job.empty() ? nullptr : &ua, ptr<const float>(grad_scale)),
             "flock_sc_round_adam");
}
void sc_round_adam_meta(at::TensorList learner, at::TensorList critic_job, at::TensorList actor_job,
                        at::IntArrayRef dims, at::ArrayRef<double> hyper, const optional<Tensor>& grad_scale) {
    TORCH_CHECK(!learner.empty(), "sc_round_adam: empty learner state");
    TORCH_CHECK(!critic_job.empty() || !actor_job.empty(), "sc_round_adam: neither a critic nor an actor phase");
    sc_round_checks(learner, critic_job, dims, hyper, "critic_job");
    sc_round_checks(learner, actor_job, dims, hyper, "actor_job");
}

// learn() prologue without a snapshot (flock_sc_prep): *agent_out = agent; idx[r] = Philox(seed, counter, r) mod rows
void sc_prep_checks(const Tensor& agent_out, const optional<Tensor>& idx, int64_t rows) {
    if (any_sym(agent_out, idx)) return;
    shaped(agent_out, "agent_out", at::kLong, {1}, agent_out);
    if (idx) {
        dense(*idx, "idx", at::kLong, agent_out);
        TORCH_CHECK(idx->dim() == 1 && idx->numel() >= 1 && rows >= 1, "sc_prep: idx [B] and rows >= 1");
    }
}
void sc_prep_hip(const Tensor& agent_out, const optional<Tensor>& idx, int64_t rows, int64_t seed, int64_t counter,
                 int64_t agent) {
    hip_only(agent_out, "sc_prep");
    sc_prep_checks(agent_out, idx, rows);
    const at::OptionalDeviceGuard g(agent_out.device());
    rc_check(flock_sc_prep(stream_of(agent_out), idx ? (int)idx->numel() : 0, rows, (uint64_t)seed, (uint64_t)counter,
                           ptr<int64_t>(idx), ptr<int64_t>(agent_out), agent),
             "flock_sc_prep");
}
void sc_prep_meta(const Tensor& agent_out, const optional<Tensor>& idx, int64_t rows, int64_t, int64_t, int64_t) {
    sc_prep_checks(agent_out, idx, rows);
}

// ------------------------------------------------------------------------------------------------------- sc_act
// obs [rows, A, in] f32 contiguous; actors: the agent-major actor buffer [A * stride] (stride = numel / A);
// actions [rows, A, 2]; ou_state / noise [rows, A, 2] (both or neither)
void sc_act_checks(const Tensor& obs, const Tensor& actors, const Tensor& actions, const optional<Tensor>& ou,
                   const optional<Tensor>& noise, int64_t fc1, int64_t fc2) {
    TORCH_CHECK(ou.has_value() == noise.has_value(), "sc_act: ou_state and noise go together");
    if (any_sym(obs, actors, actions, ou, noise)) return;
    TORCH_CHECK(obs.dim() == 3, "sc_act: obs must be [rows, n_agents, in_dim], got ", obs.sizes());
    const int64_t R = obs.size(0), A = obs.size(1), n = obs.size(2);
    dense(obs, "obs", at::kFloat, obs);
    dense(actors, "actors", at::kFloat, obs);
    TORCH_CHECK(A >= 1 && actors.numel() % A == 0, "sc_act: actors must hold n_agents equal blocks");
    TORCH_CHECK(n >= 1 && n <= 16 && fc1 >= 8 && fc1 % 8 == 0 && fc2 >= 1 && fc2 <= 320,
                "sc_act: needs 1 <= in_dim <= 16, fc1 a multiple of 8, 1 <= fc2 <= 320");
    shaped(actions, "actions", at::kFloat, {R, A, 2}, obs);
    if (ou) {
        shaped(*ou, "ou_state", at::kFloat, {R, A, 2}, obs);
        shaped(*noise, "noise", at::kFloat, {R, A, 2}, obs);
    }
}
void sc_act_hip(const Tensor& obs, const Tensor& actors, const Tensor& actions, const optional<Tensor>& ou,
                const optional<Tensor>& noise, int64_t fc1, int64_t fc2, double theta, double dt,
                double sigma_sqrt_dt) {
    hip_only(obs, "sc_act");
    sc_act_checks(obs, actors, actions, ou, noise, fc1, fc2);
    const at::OptionalDeviceGuard g(obs.device());
    rc_check(flock_sc_act(stream_of(obs), obs.size(0), (int)obs.size(1), (int)obs.size(2), (int)fc1, (int)fc2,
                          ptr<const float>(obs), ptr<const float>(actors), actors.numel() / obs.size(1),
                          ptr<float>(actions), ptr<float>(ou), ptr<const float>(noise), (float)theta, (float)dt,
                          (float)sigma_sqrt_dt),
             "flock_sc_act");
}
void sc_act_meta(const Tensor& obs, const Tensor& actors, const Tensor& actions, const optional<Tensor>& ou,
                 const optional<Tensor>& noise, int64_t fc1, int64_t fc2, double, double, double) {
    sc_act_checks(obs, actors, actions, ou, noise, fc1, fc2);
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(flock, m) {
    m.def(
        "adam_step(Tensor(a!) param, Tensor grad, Tensor(b!) exp_avg, Tensor(c!) exp_avg_sq, Tensor step, "
        "Tensor? grad_scale, Tensor(d!)? target, float lr, float beta1=0.9, float beta2=0.999, float eps=1e-08, "
        "float tau=0.0, int target_mode=0) -> ()");
    m.def("soft_update(Tensor(a!) target, Tensor src, float tau, int form=0) -> ()");
    m.def("grad_norm(Tensor grad, Tensor(a!) partial, Tensor(b!) out, float max_norm) -> ()");
    m.def("gru_cell_fwd(Tensor gi, Tensor gh, Tensor h, Tensor(a!) hout, Tensor(b!)? ws) -> ()");
    m.def("gru_cell_bwd(Tensor dhout, Tensor h, Tensor ws, Tensor(a!) dgi, Tensor(b!) dgh, Tensor(c!) dh) -> ()");
    m.def("gru_seq_fwd(Tensor gi, Tensor w_hh, Tensor b_hh, Tensor keep, Tensor(a!) hs, Tensor(b!)? ws) -> ()");
    m.def(
        "gru_seq_bwd(Tensor dhs, Tensor hs, Tensor ws, Tensor w_hh, Tensor keep, Tensor(a!) dgi, Tensor(b!) dw_hh, "
        "Tensor(c!) db_hh) -> ()");
    m.def(
        "gru_seq_q_fwd(Tensor gi, Tensor w_hh, Tensor b_hh, Tensor w_q, Tensor b_q, Tensor keep, Tensor(a!)? hs, "
        "Tensor(b!)? ws, Tensor(c!) q) -> ()");
    m.def(
        "gru_seq_q_bwd(Tensor dq, Tensor hs, Tensor ws, Tensor w_hh, Tensor w_q, Tensor keep, Tensor(a!) dgi, "
        "Tensor(b!) dw_hh, Tensor(c!) db_hh, Tensor(d!) dw_q, Tensor(e!) db_q) -> ()");
    m.def(
        "vdn_feat_fwd(Tensor x, Tensor w1, Tensor b1, Tensor w2, Tensor b2, Tensor w_ih, Tensor b_ih, "
        "Tensor(a!)? y1, Tensor(b!)? y2, Tensor(c!) gi) -> ()");
    m.def(
        "vdn_feat_bwd(Tensor x, Tensor w2, Tensor w_ih, Tensor y1, Tensor y2, Tensor dgi, Tensor(a!) dw1, "
        "Tensor(b!) db1, Tensor(c!) dw2, Tensor(d!) db2, Tensor(e!) dw_ih, Tensor(f!) db_ih) -> ()");
    m.def("gather_rows(Tensor src, Tensor idx, Tensor(a!) dst) -> ()");
    m.def("scatter_rows(Tensor src, Tensor idx, Tensor(a!) dst) -> ()");
    m.def("ring_store(Tensor[] src, Tensor(a!)[] dst, int[] kind, int start) -> ()");
    m.def(
        "sc_prep_snapshot(Tensor[] ring, Tensor(a!)[] staging, Tensor(b!) agent_out, Tensor(c!)? idx_out, int rows, "
        "int seed, int counter, int agent) -> ()");
    // sc_round / sc_round_adam mark every tensor of each list mutable (read-only replay rows and staging included)
    // and give each list one alias set; the data-parallel bucket is viewed from two lists (learner[1] and job[9]).
    // They are eager / HIP-graph ops: not for functionalization or torch.compile (which would need exact per-tensor
    // write sets and one alias annotation for the shared bucket).
    m.def(
        "sc_round(Tensor(a!)[] learner, Tensor(b!)[] critic_job, Tensor(c!)[] actor_job, int[] dims, "
        "float[] hyper) -> ()");
    m.def(
        "sc_round_adam(Tensor(a!)[] learner, Tensor(b!)[] critic_job, Tensor(c!)[] actor_job, int[] dims, "
        "float[] hyper, Tensor? grad_scale) -> ()");
    m.def("sc_prep(Tensor(a!) agent_out, Tensor(b!)? idx, int rows, int seed, int counter, int agent) -> ()");
    // the workspace floats one shared-critic job needs (flock_sc_workspace_floats; no tensors: a CatchAll kernel)
    m.def("sc_workspace_floats(int B, int in_dim, int n_actions, int fc1, int fc2) -> int",
          [](int64_t B, int64_t in_dim, int64_t na, int64_t fc1, int64_t fc2) -> int64_t {
              TORCH_CHECK(B >= 1 && in_dim >= 1 && na >= 1 && fc1 >= 1 && fc2 >= 1, "sc_workspace_floats: sizes >= 1");
              return flock_sc_workspace_floats((int)B, (int)in_dim, (int)na, (int)fc1, (int)fc2);
          });
    m.def(
        "sc_act(Tensor obs, Tensor actors, Tensor(a!) actions, Tensor(b!)? ou_state, Tensor? noise, int fc1, int fc2, "
        "float theta, float dt, float sigma_sqrt_dt) -> ()");
}

TORCH_LIBRARY_IMPL(flock, CUDA, m) {
    m.impl("adam_step", &adam_step_hip);
    m.impl("soft_update", &soft_update_hip);
    m.impl("grad_norm", &grad_norm_hip);
    m.impl("gru_cell_fwd", &gru_cell_fwd_hip);
    m.impl("gru_cell_bwd", &gru_cell_bwd_hip);
    m.impl("gru_seq_fwd", &gru_seq_fwd_hip);
    m.impl("gru_seq_bwd", &gru_seq_bwd_hip);
    m.impl("gru_seq_q_fwd", &gru_seq_q_fwd_hip);
    m.impl("gru_seq_q_bwd", &gru_seq_q_bwd_hip);
    m.impl("vdn_feat_fwd", &vdn_feat_fwd_hip);
    m.impl("vdn_feat_bwd", &vdn_feat_bwd_hip);
    m.impl("gather_rows", &gather_rows_hip);
    m.impl("scatter_rows", &scatter_rows_hip);
    m.impl("ring_store", &ring_store_hip);
    m.impl("sc_prep_snapshot", &sc_prep_snapshot_hip);
    m.impl("sc_round", &sc_round_hip);
    m.impl("sc_round_adam", &sc_round_adam_hip);
    m.impl("sc_prep", &sc_prep_hip);
    m.impl("sc_act", &sc_act_hip);
}

TORCH_LIBRARY_IMPL(flock, Meta, m) {
    m.impl("adam_step", &adam_step_meta);
    m.impl("soft_update", &soft_update_meta);
    m.impl("grad_norm", &grad_norm_meta);
    m.impl("gru_cell_fwd", &gru_cell_fwd_meta);
    m.impl("gru_cell_bwd", &gru_cell_bwd_meta);
    m.impl("gru_seq_fwd", &gru_seq_fwd_meta);
    m.impl("gru_seq_bwd", &gru_seq_bwd_meta);
    m.impl("gru_seq_q_fwd", &gru_seq_q_fwd_meta);
    m.impl("gru_seq_q_bwd", &gru_seq_q_bwd_meta);
    m.impl("vdn_feat_fwd", &vdn_feat_fwd_meta);
    m.impl("vdn_feat_bwd", &vdn_feat_bwd_meta);
    m.impl("gather_rows", &gather_rows_meta);
    m.impl("scatter_rows", &scatter_rows_meta);
    m.impl("ring_store", &ring_store_meta);
    m.impl("sc_prep_snapshot", &sc_prep_snapshot_meta);
    m.impl("sc_round", &sc_round_meta);
    m.impl("sc_round_adam", &sc_round_adam_meta);
    m.impl("sc_prep", &sc_prep_meta);
    m.impl("sc_act", &sc_act_meta);
}
