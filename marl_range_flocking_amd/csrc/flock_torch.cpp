// flock_torch.cpp — PyTorch custom ops over the C ABI (include/flock_amd.h): torch.ops.flock.*
//
// The schemas of SURVEY.md 8(b): every state or output buffer the step writes is a mutable alias argument
// (Tensor(a!)), as the reference mutates self.positions / self.headings in place (gym_flock_v2.py:329,350); the ops
// return nothing and enqueue on the current HIP stream without synchronising. Meta kernels run the same checks
// with no launch, so the ops trace under FakeTensor / torch.compile. Errors are TORCH_CHECKs (Python RuntimeError),
// with the reference's own message for k + 1 > N (torch.topk, gym_flock_v2.py:147).
//
//   flock::step_v2           gym_flock_v2.py:71-83
//   flock::step_uw           gym_flock_uw.py:69-81
//   flock::rollout_uw        K step_uw calls in one (the random-action rollout regime; config 2: one launch)
//   flock::step_uw_discrete  gym_flock_uw_discrete.py:110-122
//   flock::step_flock        gym_flock.py:48-60
//   flock::step_v2_store     step_v2 + the training loop's replay insert in the same launch (store_transitions,
//                            maddpg_shared_critic/utils.py:47-54; add_record, maddpg_official_rnn/memory_rnn.py:53-67)
//   flock::step_uw_discrete_store  step_uw_discrete + the VDN team transition (memory.put, vdn/train_flock.py:102)
//   flock::knn               _computePeriodicDistances :135-151 / _computeDistances :155-175 (functional)
//   flock::reset             reset() :85-108 and siblings (bounded draws + repair, flock_reset_ext)
#include <ATen/ATen.h>
#include <ATen/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "flock_amd.h"

namespace {

using at::Tensor;
using c10::optional;

void check_k(int64_t N, int64_t k) { TORCH_CHECK(k >= 1 && k + 1 <= N, "selected index k out of range"); }

// pos [E, N, 2] f32 on a HIP device; returns (E, N)
std::pair<int64_t, int64_t> dims(const Tensor& pos) {
    TORCH_CHECK(pos.dim() == 3 && pos.size(2) == 2, "pos must be [E, N, 2], got ", pos.sizes());
    return {pos.size(0), pos.size(1)};
}

void need(const Tensor& t, const char* name, at::ScalarType dtype, at::IntArrayRef shape, const Tensor& like) {
    TORCH_CHECK(t.device() == like.device(), name, " must be on ", like.device(), ", got ", t.device());
    TORCH_CHECK(t.scalar_type() == dtype, name, " must be ", dtype, ", got ", t.scalar_type());
    TORCH_CHECK(t.sizes() == shape, name, " must have shape ", shape, ", got ", t.sizes());
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void opt(const optional<Tensor>& t, const char* name, at::ScalarType dtype, at::IntArrayRef shape,
         const Tensor& like) {
    if (t.has_value()) need(*t, name, dtype, shape, like);
}

template <typename T>
T* ptr(const optional<Tensor>& t) {
    return t.has_value() ? static_cast<T*>(t->data_ptr()) : nullptr;
}

template <typename T>
T* ptr(const Tensor& t) {
    return static_cast<T*>(t.data_ptr());
}

void* stream_of(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void rc_check(int rc, const char* fn) { TORCH_CHECK(rc == 0, fn, ": ", flock_last_error()); }

bool on_hip(const Tensor& t) { return t.device().is_cuda(); }

// FlockStepExt.launches: the step as that many back-to-back launches over consecutive env ranges (same results)
int launch_count(int64_t launches) {
    TORCH_CHECK(launches >= 1 && launches <= 64, "launches must be in [1, 64], got ", launches);
    return (int)launches;
}

// ----------------------------------------------------------------------------------------------------- step_v2
void step_v2_checks(const Tensor& pos, const Tensor& heading, const Tensor& action, const Tensor& vel,
                    const Tensor& dnn, const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done,
                    const Tensor& any_done, const optional<Tensor>& seeds, int64_t k) {
    auto [E, N] = dims(pos);
    check_k(N, k);
    need(pos, "pos", at::kFloat, {E, N, 2}, pos);
    need(heading, "heading", at::kFloat, {E, N}, pos);
    need(action, "action", at::kFloat, {E, N, 2}, pos);
    need(vel, "vel", at::kFloat, {E, N, 2}, pos);
    need(dnn, "dnn", at::kFloat, {E, N, k}, pos);
    opt(nn_idx, "nn_idx", at::kLong, {E, N, k}, pos);
    need(reward, "reward", at::kFloat, {E, N}, pos);
    need(done, "done", at::kBool, {E, N}, pos);
    need(any_done, "any_done", at::kBool, {E}, pos);
    opt(seeds, "seeds", at::kShort, {E, N, k}, pos);
}

void step_v2_hip(const Tensor& pos, const Tensor& heading, const Tensor& action, const Tensor& vel,
                 const Tensor& dnn, const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done,
                 const Tensor& any_done, const optional<Tensor>& seeds, int64_t k, double box, double sensor_range,
                 double collision_distance, double dt, double v_min, double v_max, bool periodic,
                 bool rigid_boundary, int64_t launches, bool normalize_distance) {
    TORCH_CHECK(on_hip(pos), "flock ops run on a HIP device only (no CPU fallback); got ", pos.device());
    const at::OptionalDeviceGuard guard(pos.device());
    step_v2_checks(pos, heading, action, vel, dnn, nn_idx, reward, done, any_done, seeds, k);
    FlockStepExt ext{nullptr, ptr<uint16_t>(seeds), launch_count(launches), normalize_distance ? 1 : 0};
    rc_check(flock_step_v2_ext(stream_of(pos), (int)pos.size(0), (int)pos.size(1), (int)k, (float)box,
                               (float)sensor_range, (float)collision_distance, (float)dt, (float)v_min,
                               (float)v_max, periodic, rigid_boundary, ptr<float>(pos), ptr<float>(heading),
                               ptr<const float>(action), ptr<float>(vel), ptr<float>(dnn), ptr<int64_t>(nn_idx),
                               ptr<float>(reward), ptr<uint8_t>(done), ptr<uint8_t>(any_done), &ext),
             "flock_step_v2");
}

void step_v2_meta(const Tensor& pos, const Tensor& heading, const Tensor& action, const Tensor& vel,
                  const Tensor& dnn, const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done,
                  const Tensor& any_done, const optional<Tensor>& seeds, int64_t k, double, double, double, double,
                  double, double, bool, bool, int64_t launches, bool) {
    launch_count(launches);
    step_v2_checks(pos, heading, action, vel, dnn, nn_idx, reward, done, any_done, seeds, k);
}

// ----------------------------------------------------------------------------------------------------- step_uw
void step_uw_checks(const Tensor& pos, const Tensor& heading, const Tensor& prev_heading, const Tensor& action,
                    const Tensor& mem_in, const Tensor& mem_out, const Tensor& vel, const Tensor& dnn,
                    const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done,
                    const Tensor& any_done, const optional<Tensor>& seeds, int64_t k) {
    auto [E, N] = dims(pos);
    check_k(N, k);
    need(pos, "pos", at::kFloat, {E, N, 2}, pos);
    need(heading, "heading", at::kFloat, {E, N}, pos);
    need(prev_heading, "prev_heading", at::kFloat, {E, N}, pos);
    need(action, "action", at::kFloat, {E, N, 2}, pos);
    need(mem_in, "mem_in", at::kFloat, {E, N, 4, k}, pos);
    need(mem_out, "mem_out", at::kFloat, {E, N, 4, k}, pos);
    need(vel, "vel", at::kFloat, {E, N, 2}, pos);
    need(dnn, "dnn", at::kFloat, {E, N, k}, pos);
    opt(nn_idx, "nn_idx", at::kLong, {E, N, k}, pos);
    need(reward, "reward", at::kFloat, {E, N}, pos);
    need(done, "done", at::kBool, {E, N}, pos);
    need(any_done, "any_done", at::kBool, {E}, pos);
    opt(seeds, "seeds", at::kShort, {E, N, k}, pos);
}

void step_uw_hip(const Tensor& pos, const Tensor& heading, const Tensor& prev_heading, const Tensor& action,
                 const Tensor& mem_in, const Tensor& mem_out, const Tensor& vel, const Tensor& dnn,
                 const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done, const Tensor& any_done,
                 const optional<Tensor>& seeds, int64_t k, double box, double sensor_range,
                 double collision_distance, double dt, bool rigid_boundary, int64_t launches,
                 bool normalize_distance) {
    TORCH_CHECK(on_hip(pos), "flock ops run on a HIP device only (no CPU fallback); got ", pos.device());
    const at::OptionalDeviceGuard guard(pos.device());
    step_uw_checks(pos, heading, prev_heading, action, mem_in, mem_out, vel, dnn, nn_idx, reward, done, any_done,
                   seeds, k);
    FlockStepExt ext{nullptr, ptr<uint16_t>(seeds), launch_count(launches), normalize_distance ? 1 : 0};
    rc_check(flock_step_uw_ext(stream_of(pos), (int)pos.size(0), (int)pos.size(1), (int)k, (float)box,
                               (float)sensor_range, (float)collision_distance, (float)dt, rigid_boundary,
                               ptr<float>(pos), ptr<const float>(heading), ptr<float>(prev_heading),
                               ptr<const float>(action), ptr<const float>(mem_in), ptr<float>(mem_out),
                               ptr<float>(vel), ptr<float>(dnn), ptr<int64_t>(nn_idx), ptr<float>(reward),
                               ptr<uint8_t>(done), ptr<uint8_t>(any_done), &ext),
             "flock_step_uw");
}

void step_uw_meta(const Tensor& pos, const Tensor& heading, const Tensor& prev_heading, const Tensor& action,
                  const Tensor& mem_in, const Tensor& mem_out, const Tensor& vel, const Tensor& dnn,
                  const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done, const Tensor& any_done,
                  const optional<Tensor>& seeds, int64_t k, double, double, double, double, bool, int64_t launches,
                  bool) {
    launch_count(launches);
    step_uw_checks(pos, heading, prev_heading, action, mem_in, mem_out, vel, dnn, nn_idx, reward, done, any_done,
                   seeds, k);
}

// -------------------------------------------------------------------------------------------------- rollout_uw
// K steps of step_uw in one call (flock_rollout_uw): actions [K, E, N, 2]; per-step outputs obs_out [K, E, N, 4, k],
// reward_out [K, E, N], done_out [K, E, N], any_done_out [K, E]; the env buffers end as after K step_uw calls
void rollout_uw_checks(const Tensor& pos, const Tensor& heading, const Tensor& prev_heading, const Tensor& actions,
                       const Tensor& mem_in, const Tensor& mem_out, const Tensor& vel, const Tensor& dnn,
                       const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done, const Tensor& any_done,
                       const Tensor& obs_out, const Tensor& reward_out, const Tensor& done_out,
                       const Tensor& any_done_out, const optional<Tensor>& seeds, int64_t k) {
    TORCH_CHECK(actions.dim() == 4, "actions must be [K, E, N, 2], got ", actions.sizes());
    const int64_t K = actions.size(0);
    auto [E, N] = dims(pos);
    step_uw_checks(pos, heading, prev_heading, actions[0], mem_in, mem_out, vel, dnn, nn_idx, reward, done, any_done,
                   seeds, k);
    need(actions, "actions", at::kFloat, {K, E, N, 2}, pos);
    need(obs_out, "obs_out", at::kFloat, {K, E, N, 4, k}, pos);
    need(reward_out, "reward_out", at::kFloat, {K, E, N}, pos);
    need(done_out, "done_out", at::kBool, {K, E, N}, pos);
    need(any_done_out, "any_done_out", at::kBool, {K, E}, pos);
}

void rollout_uw_hip(const Tensor& pos, const Tensor& heading, const Tensor& prev_heading, const Tensor& actions,
                    const Tensor& mem_in, const Tensor& mem_out, const Tensor& vel, const Tensor& dnn,
                    const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done, const Tensor& any_done,
                    const Tensor& obs_out, const Tensor& reward_out, const Tensor& done_out,
                    const Tensor& any_done_out, const optional<Tensor>& seeds, int64_t k, double box,
                    double sensor_range, double collision_distance, double dt, bool rigid_boundary,
                    bool normalize_distance) {
    TORCH_CHECK(on_hip(pos), "flock ops run on a HIP device only (no CPU fallback); got ", pos.device());
    const at::OptionalDeviceGuard guard(pos.device());
    rollout_uw_checks(pos, heading, prev_heading, actions, mem_in, mem_out, vel, dnn, nn_idx, reward, done, any_done,
                      obs_out, reward_out, done_out, any_done_out, seeds, k);
    FlockStepExt ext{nullptr, ptr<uint16_t>(seeds), 1, normalize_distance ? 1 : 0};
    rc_check(flock_rollout_uw(stream_of(pos), (int)actions.size(0), (int)pos.size(0), (int)pos.size(1), (int)k,
                              (float)box, (float)sensor_range, (float)collision_distance, (float)dt, rigid_boundary,
                              ptr<float>(pos), ptr<const float>(heading), ptr<float>(prev_heading),
                              ptr<const float>(actions), ptr<const float>(mem_in), ptr<float>(mem_out), ptr<float>(vel),
                              ptr<float>(dnn), ptr<int64_t>(nn_idx), ptr<float>(reward), ptr<uint8_t>(done),
                              ptr<uint8_t>(any_done), ptr<float>(obs_out), ptr<float>(reward_out),
                              ptr<uint8_t>(done_out), ptr<uint8_t>(any_done_out), &ext),
             "flock_rollout_uw");
}

void rollout_uw_meta(const Tensor& pos, const Tensor& heading, const Tensor& prev_heading, const Tensor& actions,
                     const Tensor& mem_in, const Tensor& mem_out, const Tensor& vel, const Tensor& dnn,
                     const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done, const Tensor& any_done,
                     const Tensor& obs_out, const Tensor& reward_out, const Tensor& done_out,
                     const Tensor& any_done_out, const optional<Tensor>& seeds, int64_t k, double, double, double,
                     double, bool, bool) {
    rollout_uw_checks(pos, heading, prev_heading, actions, mem_in, mem_out, vel, dnn, nn_idx, reward, done, any_done,
                      obs_out, reward_out, done_out, any_done_out, seeds, k);
}

// -------------------------------------------------------------------------------------------- step_uw_discrete
void step_uwd_checks(const Tensor& pos, const Tensor& heading, const Tensor& prev_heading, const Tensor& action_id,
                     const optional<Tensor>& noise, const Tensor& table, const Tensor& vel, const Tensor& dnn,
                     const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done,
                     const Tensor& any_done, const Tensor& status, const optional<Tensor>& seeds, int64_t k) {
    auto [E, N] = dims(pos);
    check_k(N, k);
    need(pos, "pos", at::kFloat, {E, N, 2}, pos);
    need(heading, "heading", at::kFloat, {E, N}, pos);
    need(prev_heading, "prev_heading", at::kFloat, {E, N}, pos);
    need(action_id, "action_id", at::kLong, {E, N}, pos);
    opt(noise, "noise", at::kFloat, {E, N, 2}, pos);
    TORCH_CHECK(table.dim() == 2 && table.size(1) == 2, "table must be [n_actions, 2]");
    need(table, "table", at::kFloat, table.sizes(), pos);
    need(vel, "vel", at::kFloat, {E, N, 2}, pos);
    need(dnn, "dnn", at::kFloat, {E, N, k}, pos);
    opt(nn_idx, "nn_idx", at::kLong, {E, N, k}, pos);
    need(reward, "reward", at::kFloat, {E, N}, pos);
    need(done, "done", at::kBool, {E, N}, pos);
    need(any_done, "any_done", at::kBool, {E}, pos);
    need(status, "status", at::kInt, {1}, pos);
    opt(seeds, "seeds", at::kShort, {E, N, k}, pos);
}

void step_uwd_hip(const Tensor& pos, const Tensor& heading, const Tensor& prev_heading, const Tensor& action_id,
                  const optional<Tensor>& noise, const Tensor& table, const Tensor& vel, const Tensor& dnn,
                  const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done, const Tensor& any_done,
                  const Tensor& status, const optional<Tensor>& seeds, int64_t k, double box, double sensor_range,
                  double collision_distance, double dt, double v_max, bool rigid_boundary, double noise_std,
                  int64_t seed, int64_t rng_offset, int64_t launches, bool normalize_distance) {
    TORCH_CHECK(on_hip(pos), "flock ops run on a HIP device only (no CPU fallback); got ", pos.device());
    const at::OptionalDeviceGuard guard(pos.device());
    step_uwd_checks(pos, heading, prev_heading, action_id, noise, table, vel, dnn, nn_idx, reward, done, any_done,
                    status, seeds, k);
    FlockStepExt ext{nullptr, ptr<uint16_t>(seeds), launch_count(launches), normalize_distance ? 1 : 0};
    rc_check(flock_step_uw_discrete_ext(
                 stream_of(pos), (int)pos.size(0), (int)pos.size(1), (int)k, (float)box, (float)sensor_range,
                 (float)collision_distance, (float)dt, (float)v_max, rigid_boundary, ptr<float>(pos),
                 ptr<float>(heading), ptr<float>(prev_heading), ptr<const int64_t>(action_id),
                 ptr<const float>(noise), (float)noise_std, (uint64_t)seed, (uint64_t)rng_offset,
                 ptr<const float>(table), (int)table.size(0), ptr<float>(vel), ptr<float>(dnn),
                 ptr<int64_t>(nn_idx), ptr<float>(reward), ptr<uint8_t>(done), ptr<uint8_t>(any_done),
                 ptr<int>(status), &ext),
             "flock_step_uw_discrete");
}

void step_uwd_meta(const Tensor& pos, const Tensor& heading, const Tensor& prev_heading, const Tensor& action_id,
                   const optional<Tensor>& noise, const Tensor& table, const Tensor& vel, const Tensor& dnn,
                   const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done, const Tensor& any_done,
                   const Tensor& status, const optional<Tensor>& seeds, int64_t k, double, double, double, double,
                   double, bool, double, int64_t, int64_t, int64_t launches, bool) {
    launch_count(launches);
    step_uwd_checks(pos, heading, prev_heading, action_id, noise, table, vel, dnn, nn_idx, reward, done, any_done,
                    status, seeds, k);
}

// -------------------------------------------------------------------------------------------------- step_flock
void step_flock_checks(const Tensor& pos, const Tensor& vel, const Tensor& action, const Tensor& mem_in,
                       const Tensor& mem_out, const Tensor& dnn, const optional<Tensor>& nn_idx,
                       const Tensor& reward, const Tensor& done, const Tensor& any_done,
                       const optional<Tensor>& seeds, int64_t k) {
    auto [E, N] = dims(pos);
    check_k(N, k);
    need(pos, "pos", at::kFloat, {E, N, 2}, pos);
    need(vel, "vel", at::kFloat, {E, N, 2}, pos);
    need(action, "action", at::kFloat, {E, N, 2}, pos);
    need(mem_in, "mem_in", at::kFloat, {E, N, 4, k}, pos);
    need(mem_out, "mem_out", at::kFloat, {E, N, 4, k}, pos);
    need(dnn, "dnn", at::kFloat, {E, N, k}, pos);
    opt(nn_idx, "nn_idx", at::kLong, {E, N, k}, pos);
    need(reward, "reward", at::kFloat, {E, N}, pos);
    need(done, "done", at::kBool, {E, N}, pos);
    need(any_done, "any_done", at::kBool, {E}, pos);
    opt(seeds, "seeds", at::kShort, {E, N, k}, pos);
}

void step_flock_hip(const Tensor& pos, const Tensor& vel, const Tensor& action, const Tensor& mem_in,
                    const Tensor& mem_out, const Tensor& dnn, const optional<Tensor>& nn_idx, const Tensor& reward,
                    const Tensor& done, const Tensor& any_done, const optional<Tensor>& seeds, int64_t k,
                    double box, double collision_distance, double dt, bool rigid_boundary, int64_t launches,
                    bool normalize_distance) {
    TORCH_CHECK(on_hip(pos), "flock ops run on a HIP device only (no CPU fallback); got ", pos.device());
    const at::OptionalDeviceGuard guard(pos.device());
    step_flock_checks(pos, vel, action, mem_in, mem_out, dnn, nn_idx, reward, done, any_done, seeds, k);
    FlockStepExt ext{nullptr, ptr<uint16_t>(seeds), launch_count(launches), normalize_distance ? 1 : 0};
    rc_check(flock_step_flock_ext(stream_of(pos), (int)pos.size(0), (int)pos.size(1), (int)k, (float)box,
                                  (float)collision_distance, (float)dt, rigid_boundary, ptr<float>(pos),
                                  ptr<float>(vel), ptr<const float>(action), ptr<const float>(mem_in),
                                  ptr<float>(mem_out), ptr<float>(dnn), ptr<int64_t>(nn_idx), ptr<float>(reward),
                                  ptr<uint8_t>(done), ptr<uint8_t>(any_done), &ext),
             "flock_step_flock");
}

void step_flock_meta(const Tensor& pos, const Tensor& vel, const Tensor& action, const Tensor& mem_in,
                     const Tensor& mem_out, const Tensor& dnn, const optional<Tensor>& nn_idx, const Tensor& reward,
                     const Tensor& done, const Tensor& any_done, const optional<Tensor>& seeds, int64_t k, double,
                     double, double, bool, int64_t launches, bool) {
    launch_count(launches);
    step_flock_checks(pos, vel, action, mem_in, mem_out, dnn, nn_idx, reward, done, any_done, seeds, k);
}


// ------------------------------------------------------------------------------------ fused replay insert (ring)
// ring = [state, action, reward, new_state, terminal] device rings ([capacity, ...] f32), the optional record copies
// actor_state / actor_new_state, prev_obs [E, N, k] (the observation before the step); meta = [start, skip, group,
// store_done, action_ids, env_done] (FlockRing, include/flock_amd.h)
FlockRing ring_of(const Tensor& pos, at::TensorList ring, const optional<Tensor>& actor_state,
                  const optional<Tensor>& actor_new_state, const Tensor& prev_obs, at::IntArrayRef meta, int64_t k) {
    // traced with symbolic sizes (AOT dispatch, dynamic shapes): no concrete sizes to check (the HIP wrapper does)
    auto sym = [](const Tensor& t) { return t.defined() && t.unsafeGetTensorImpl()->has_symbolic_sizes_strides(); };
    bool any = sym(pos) || sym(prev_obs) || (actor_state && sym(*actor_state)) ||
               (actor_new_state && sym(*actor_new_state));
    for (const Tensor& t : ring) any = any || sym(t);
    if (any) return FlockRing{};
    auto [E, N] = dims(pos);
    TORCH_CHECK(ring.size() == 5, "ring must be [state, action, reward, new_state, terminal]");
    TORCH_CHECK(meta.size() == 6, "ring_meta must be [start, skip, group, store_done, action_ids, env_done]");
    const int64_t start = meta[0], skip = meta[1], group = meta[2];
    const bool ids = meta[4] != 0, env_done = meta[5] != 0;
    TORCH_CHECK(group == 1 || group == N, "ring group must be 1 (a row per agent) or N (a row per env)");
    TORCH_CHECK(!env_done || group == N, "env_done needs a row per env (group = N)");
    TORCH_CHECK(ring[0].dim() >= 1, "ring fields must be [capacity, ...]");
    const int64_t cap = ring[0].size(0), units = group == 1 ? E * N : E;
    TORCH_CHECK(skip >= 0 && units - skip <= cap && start >= 0 && start < cap,
                "ring: need 0 <= skip, rows - skip <= capacity and 0 <= start < capacity");
    const char* names[5] = {"ring state", "ring action", "ring reward", "ring new_state", "ring terminal"};
    const int64_t w[5] = {group * k, group * (ids ? 1 : 2), group, group * k, env_done ? 1 : group};
    for (int i = 0; i < 5; ++i) {
        TORCH_CHECK(ring[i].device() == pos.device() && ring[i].scalar_type() == at::kFloat &&
                        ring[i].is_contiguous() && ring[i].dim() >= 1 && ring[i].size(0) == cap &&
                        ring[i].numel() == cap * w[i],
                    names[i], " must be a contiguous f32 [", cap, ", ", w[i], "] ring on ", pos.device());
    }
    const optional<Tensor>* extra[2] = {&actor_state, &actor_new_state};
    for (const optional<Tensor>* t : extra)
        if (t->has_value())
            TORCH_CHECK((*t)->device() == pos.device() && (*t)->scalar_type() == at::kFloat &&
                            (*t)->is_contiguous() && (*t)->numel() == cap * group * k,
                        "ring actor_state / actor_new_state must be contiguous f32 [", cap, ", ", group * k, "]");
    need(prev_obs, "prev_obs", at::kFloat, {E, N, k}, pos);
    FlockRing r{};
    r.state = ptr<float>(ring[0]);
    r.action = ptr<float>(ring[1]);
    r.reward = ptr<float>(ring[2]);
    r.new_state = ptr<float>(ring[3]);
    r.terminal = ptr<float>(ring[4]);
    r.prev_obs = ptr<const float>(prev_obs);
    r.capacity = cap;
    r.start = start;
    r.skip = skip;
    r.actor_state = ptr<float>(actor_state);
    r.actor_new_state = ptr<float>(actor_new_state);
    r.group = group;
    r.store_done = meta[3] != 0;
    r.action_ids = ids;
    r.env_done = env_done;
    return r;
}

void step_v2_store_hip(const Tensor& pos, const Tensor& heading, const Tensor& action, const Tensor& vel,
                       const Tensor& dnn, const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done,
                       const Tensor& any_done, const optional<Tensor>& seeds, at::TensorList ring,
                       const optional<Tensor>& actor_state, const optional<Tensor>& actor_new_state,
                       const Tensor& prev_obs, at::IntArrayRef ring_meta, int64_t k, double box, double sensor_range,
                       double collision_distance, double dt, double v_min, double v_max, bool periodic,
                       bool rigid_boundary, int64_t launches, bool normalize_distance) {
    TORCH_CHECK(on_hip(pos), "flock ops run on a HIP device only (no CPU fallback); got ", pos.device());
    const at::OptionalDeviceGuard guard(pos.device());
    step_v2_checks(pos, heading, action, vel, dnn, nn_idx, reward, done, any_done, seeds, k);
    TORCH_CHECK(ring_meta.size() == 6 && ring_meta[4] == 0 && ring_meta[5] == 0,
                "step_v2_store: action ids / env done flags are the uw_discrete ring's");
    const FlockRing r = ring_of(pos, ring, actor_state, actor_new_state, prev_obs, ring_meta, k);
    FlockStepExt ext{&r, ptr<uint16_t>(seeds), launch_count(launches), normalize_distance ? 1 : 0};
    rc_check(flock_step_v2_ext(stream_of(pos), (int)pos.size(0), (int)pos.size(1), (int)k, (float)box,
                               (float)sensor_range, (float)collision_distance, (float)dt, (float)v_min,
                               (float)v_max, periodic, rigid_boundary, ptr<float>(pos), ptr<float>(heading),
                               ptr<const float>(action), ptr<float>(vel), ptr<float>(dnn), ptr<int64_t>(nn_idx),
                               ptr<float>(reward), ptr<uint8_t>(done), ptr<uint8_t>(any_done), &ext),
             "flock_step_v2_store");
}

void step_v2_store_meta(const Tensor& pos, const Tensor& heading, const Tensor& action, const Tensor& vel,
                        const Tensor& dnn, const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done,
                        const Tensor& any_done, const optional<Tensor>& seeds, at::TensorList ring,
                        const optional<Tensor>& actor_state, const optional<Tensor>& actor_new_state,
                        const Tensor& prev_obs, at::IntArrayRef ring_meta, int64_t k, double, double, double, double,
                        double, double, bool, bool, int64_t launches, bool) {
    launch_count(launches);
    step_v2_checks(pos, heading, action, vel, dnn, nn_idx, reward, done, any_done, seeds, k);
    ring_of(pos, ring, actor_state, actor_new_state, prev_obs, ring_meta, k);
}

void step_uwd_store_hip(const Tensor& pos, const Tensor& heading, const Tensor& prev_heading, const Tensor& action_id,
                        const optional<Tensor>& noise, const Tensor& table, const Tensor& vel, const Tensor& dnn,
                        const optional<Tensor>& nn_idx, const Tensor& reward, const Tensor& done,
                        const Tensor& any_done, const Tensor& status, const optional<Tensor>& seeds,
                        at::TensorList ring, const Tensor& prev_obs, at::IntArrayRef ring_meta, int64_t k, double box,
                        double sensor_range, double collision_distance, double dt, double v_max, bool rigid_boundary,
                        double noise_std, int64_t seed, int64_t rng_offset, int64_t launches,
                        bool normalize_distance) {
    TORCH_CHECK(on_hip(pos), "flock ops run on a HIP device only (no CPU fallback); got ", pos.device());
    const at::OptionalDeviceGuard guard(pos.device());
    step_uwd_checks(pos, heading, prev_heading, action_id, noise, table, vel, dnn, nn_idx, reward, done, any_done,
                    status, seeds, k);
    const FlockRing r = ring_of(pos, ring, c10::nullopt, c10::nullopt, prev_obs, ring_meta, k);
    FlockStepExt ext{&r, ptr<uint16_t>(seeds), launch_count(launches), normalize_distance ? 1 : 0};
    rc_check(flock_step_uw_discrete_ext(
                 stream_of(pos), (int)pos.size(0), (int)pos.size(1), (int)k, (float)box, (float)sensor_range,
                 (float)collision_distance, (float)dt, (float)v_max, rigid_boundary, ptr<float>(pos),
                 ptr<float>(heading), ptr<float>(prev_heading), ptr<const int64_t>(action_id),
                 ptr<const float>(noise), (float)noise_std, (uint64_t)seed, (uint64_t)rng_offset,
                 ptr<const float>(table), (int)table.size(0), ptr<float>(vel), ptr<float>(dnn),
                 ptr<int64_t>(nn_idx), ptr<float>(reward), ptr<uint8_t>(done), ptr<uint8_t>(any_done),
                 ptr<int>(status), &ext),
             "flock_step_uw_discrete_store");
}

void step_uwd_store_meta(const Tensor& pos, const Tensor& heading, const Tensor& prev_heading,
                         const Tensor& action_id, const optional<Tensor>& noise, const Tensor& table,
                         const Tensor& vel, const Tensor& dnn, const optional<Tensor>& nn_idx, const Tensor& reward,
                         const Tensor& done, const Tensor& any_done, const Tensor& status,
                         const optional<Tensor>& seeds, at::TensorList ring, const Tensor& prev_obs,
                         at::IntArrayRef ring_meta, int64_t k, double, double, double, double, double, bool, double,
                         int64_t, int64_t, int64_t launches, bool) {
    launch_count(launches);
    step_uwd_checks(pos, heading, prev_heading, action_id, noise, table, vel, dnn, nn_idx, reward, done, any_done,
                    status, seeds, k);
    ring_of(pos, ring, c10::nullopt, c10::nullopt, prev_obs, ring_meta, k);
}

// --------------------------------------------------------------------------------------------------------- knn
std::tuple<Tensor, Tensor> knn_alloc(const Tensor& pos, int64_t k) {
    auto [E, N] = dims(pos);
    check_k(N, k);
    TORCH_CHECK(pos.scalar_type() == at::kFloat, "pos must be float32, got ", pos.scalar_type());
    return {at::empty({E, N, k}, pos.options()), at::empty({E, N, k}, pos.options().dtype(at::kLong))};
}

std::tuple<Tensor, Tensor> knn_hip(const Tensor& pos_in, int64_t k, double box, double sensor_range, bool periodic,
                                   bool clamp) {
    TORCH_CHECK(on_hip(pos_in), "flock ops run on a HIP device only (no CPU fallback); got ", pos_in.device());
    const at::OptionalDeviceGuard guard(pos_in.device());
    const Tensor pos = pos_in.contiguous();
    auto out = knn_alloc(pos, k);
    rc_check(flock_knn(stream_of(pos), (int)pos.size(0), (int)pos.size(1), (int)k, (float)box, (float)sensor_range,
                       periodic, clamp, ptr<const float>(pos), ptr<float>(std::get<0>(out)),
                       ptr<int64_t>(std::get<1>(out))),
             "flock_knn");
    return out;
}

std::tuple<Tensor, Tensor> knn_meta(const Tensor& pos, int64_t k, double, double, bool, bool) {
    return knn_alloc(pos, k);
}

// ------------------------------------------------------------------------------------------------------- reset
void reset_checks(const Tensor& pos, const Tensor& dnn, const optional<Tensor>& heading,
                  const optional<Tensor>& prev_heading, const optional<Tensor>& vel, const optional<Tensor>& nn_idx,
                  const optional<Tensor>& mem, const optional<Tensor>& valid, const optional<Tensor>& env_mask,
                  int64_t variant, int64_t k) {
    auto [E, N] = dims(pos);
    check_k(N, k);
    TORCH_CHECK(variant >= 0 && variant <= 3, "variant must be 0 (v2), 1 (uw), 2 (uw_discrete) or 3 (flock)");
    need(pos, "pos", at::kFloat, {E, N, 2}, pos);
    need(dnn, "dnn", at::kFloat, {E, N, k}, pos);
    opt(heading, "heading", at::kFloat, {E, N}, pos);
    opt(prev_heading, "prev_heading", at::kFloat, {E, N}, pos);
    opt(vel, "vel", at::kFloat, {E, N, 2}, pos);
    opt(nn_idx, "nn_idx", at::kLong, {E, N, k}, pos);
    opt(mem, "mem", at::kFloat, {E, N, 4, k}, pos);
    opt(valid, "valid", at::kBool, {E}, pos);
    opt(env_mask, "env_mask", at::kBool, {E}, pos);
}

void reset_hip(const Tensor& pos, const Tensor& dnn, const optional<Tensor>& heading,
               const optional<Tensor>& prev_heading, const optional<Tensor>& vel, const optional<Tensor>& nn_idx,
               const optional<Tensor>& mem, const optional<Tensor>& valid, const optional<Tensor>& env_mask,
               int64_t variant, int64_t k, double range_lo, double range_hi, double box, double sensor_range,
               double check_distance, bool rigid_boundary, int64_t max_attempts, int64_t seed, int64_t rng_offset,
               int64_t repair_rounds, bool normalize_distance) {
    TORCH_CHECK(on_hip(pos), "flock ops run on a HIP device only (no CPU fallback); got ", pos.device());
    const at::OptionalDeviceGuard guard(pos.device());
    reset_checks(pos, dnn, heading, prev_heading, vel, nn_idx, mem, valid, env_mask, variant, k);
    rc_check(flock_reset_ext2(stream_of(pos), (int)variant, (int)pos.size(0), (int)pos.size(1), (int)k,
                              (float)range_lo, (float)range_hi, (float)box, (float)sensor_range, (float)check_distance,
                              rigid_boundary, (int)max_attempts, (uint64_t)seed, (uint64_t)rng_offset,
                              ptr<const uint8_t>(env_mask), ptr<float>(pos), ptr<float>(heading),
                              ptr<float>(prev_heading), ptr<float>(vel), ptr<float>(dnn), ptr<int64_t>(nn_idx),
                              ptr<float>(mem), ptr<uint8_t>(valid), (int)repair_rounds, normalize_distance ? 1 : 0),
             "flock_reset");
}

void reset_meta(const Tensor& pos, const Tensor& dnn, const optional<Tensor>& heading,
                const optional<Tensor>& prev_heading, const optional<Tensor>& vel, const optional<Tensor>& nn_idx,
                const optional<Tensor>& mem, const optional<Tensor>& valid, const optional<Tensor>& env_mask,
                int64_t variant, int64_t k, double, double, double, double, double, bool, int64_t, int64_t, int64_t,
                int64_t, bool) {
    reset_checks(pos, dnn, heading, prev_heading, vel, nn_idx, mem, valid, env_mask, variant, k);
}

}  // namespace

TORCH_LIBRARY(flock, m) {
    m.def(
        "step_v2(Tensor(a!) pos, Tensor(b!) heading, Tensor action, Tensor(c!) vel, Tensor(d!) dnn, "
        "Tensor(e!)? nn_idx, Tensor(f!) reward, Tensor(g!) done, Tensor(h!) any_done, Tensor(i!)? seeds, int k, "
        "float box, float sensor_range, float collision_distance, float dt=0.1, float v_min=0.005, "
        "float v_max=2.5, bool periodic=True, bool rigid_boundary=False, int launches=1, "
        "bool normalize_distance=False) -> ()");
    m.def(
        "step_uw(Tensor(a!) pos, Tensor heading, Tensor(b!) prev_heading, Tensor action, Tensor mem_in, "
        "Tensor(c!) mem_out, Tensor(d!) vel, Tensor(e!) dnn, Tensor(f!)? nn_idx, Tensor(g!) reward, "
        "Tensor(h!) done, Tensor(i!) any_done, Tensor(j!)? seeds, int k, float box, float sensor_range, "
        "float collision_distance, float dt=0.1, bool rigid_boundary=False, int launches=1, "
        "bool normalize_distance=False) -> ()");
    m.def(
        "rollout_uw(Tensor(a!) pos, Tensor heading, Tensor(b!) prev_heading, Tensor actions, Tensor mem_in, "
        "Tensor(c!) mem_out, Tensor(d!) vel, Tensor(e!) dnn, Tensor(f!)? nn_idx, Tensor(g!) reward, "
        "Tensor(h!) done, Tensor(i!) any_done, Tensor(j!) obs_out, Tensor(k!) reward_out, Tensor(l!) done_out, "
        "Tensor(m!) any_done_out, Tensor(n!)? seeds, int k, float box, float sensor_range, float collision_distance, "
        "float dt=0.1, bool rigid_boundary=False, bool normalize_distance=False) -> ()");
    m.def(
        "step_uw_discrete(Tensor(a!) pos, Tensor(b!) heading, Tensor(c!) prev_heading, Tensor action_id, "
        "Tensor? noise, Tensor table, Tensor(d!) vel, Tensor(e!) dnn, Tensor(f!)? nn_idx, Tensor(g!) reward, "
        "Tensor(h!) done, Tensor(i!) any_done, Tensor(j!) status, Tensor(l!)? seeds, int k, float box, "
        "float sensor_range, float collision_distance, float dt=0.1, float v_max=2.5, bool rigid_boundary=False, "
        "float noise_std=0.1, int seed=0, int rng_offset=0, int launches=1, bool normalize_distance=False) "
        "-> ()");
    m.def(
        "step_flock(Tensor(a!) pos, Tensor(b!) vel, Tensor action, Tensor mem_in, Tensor(c!) mem_out, "
        "Tensor(d!) dnn, Tensor(e!)? nn_idx, Tensor(f!) reward, Tensor(g!) done, Tensor(h!) any_done, "
        "Tensor(i!)? seeds, int k, float box, float collision_distance, float dt=0.1, "
        "bool rigid_boundary=False, int launches=1, bool normalize_distance=False) -> ()");
    m.def(
        "step_v2_store(Tensor(a!) pos, Tensor(b!) heading, Tensor action, Tensor(c!) vel, Tensor(d!) dnn, "
        "Tensor(e!)? nn_idx, Tensor(f!) reward, Tensor(g!) done, Tensor(h!) any_done, Tensor(i!)? seeds, "
        "Tensor(j!)[] ring, Tensor(k!)? ring_actor_state, Tensor(l!)? ring_actor_new_state, Tensor prev_obs, "
        "int[] ring_meta, int k, float box, float sensor_range, float collision_distance, float dt=0.1, "
        "float v_min=0.005, float v_max=2.5, bool periodic=True, bool rigid_boundary=False, int launches=1, "
        "bool normalize_distance=False) -> ()");
    m.def(
        "step_uw_discrete_store(Tensor(a!) pos, Tensor(b!) heading, Tensor(c!) prev_heading, Tensor action_id, "
        "Tensor? noise, Tensor table, Tensor(d!) vel, Tensor(e!) dnn, Tensor(f!)? nn_idx, Tensor(g!) reward, "
        "Tensor(h!) done, Tensor(i!) any_done, Tensor(j!) status, Tensor(l!)? seeds, Tensor(m!)[] ring, "
        "Tensor prev_obs, int[] ring_meta, int k, float box, float sensor_range, float collision_distance, "
        "float dt=0.1, float v_max=2.5, bool rigid_boundary=False, float noise_std=0.1, int seed=0, "
        "int rng_offset=0, int launches=1, bool normalize_distance=False) -> ()");
    m.def(
        "knn(Tensor pos, int k, float box, float sensor_range=14.0, bool periodic=True, bool clamp=True) "
        "-> (Tensor dnn, Tensor nn_idx)");
    m.def(
        "reset(Tensor(a!) pos, Tensor(b!) dnn, Tensor(c!)? heading, Tensor(d!)? prev_heading, Tensor(e!)? vel, "
        "Tensor(f!)? nn_idx, Tensor(g!)? mem, Tensor(h!)? valid, Tensor? env_mask, int variant, int k, "
        "float range_lo, float range_hi, float box, float sensor_range, float check_distance, "
        "bool rigid_boundary=False, int max_attempts=64, int seed=0, int rng_offset=0, int repair_rounds=0, "
        "bool normalize_distance=False) -> ()");
}

TORCH_LIBRARY_IMPL(flock, CUDA, m) {  // ROCm builds of PyTorch dispatch HIP tensors under the CUDA key
    m.impl("step_v2", &step_v2_hip);
    m.impl("step_uw", &step_uw_hip);
    m.impl("rollout_uw", &rollout_uw_hip);
    m.impl("step_uw_discrete", &step_uwd_hip);
    m.impl("step_flock", &step_flock_hip);
    m.impl("step_v2_store", &step_v2_store_hip);
    m.impl("step_uw_discrete_store", &step_uwd_store_hip);
    m.impl("knn", &knn_hip);
    m.impl("reset", &reset_hip);
}

TORCH_LIBRARY_IMPL(flock, Meta, m) {
    m.impl("step_v2", &step_v2_meta);
    m.impl("step_uw", &step_uw_meta);
    m.impl("rollout_uw", &rollout_uw_meta);
    m.impl("step_uw_discrete", &step_uwd_meta);
    m.impl("step_flock", &step_flock_meta);
    m.impl("step_v2_store", &step_v2_store_meta);
    m.impl("step_uw_discrete_store", &step_uwd_store_meta);
    m.impl("knn", &knn_meta);
    m.impl("reset", &reset_meta);
}
