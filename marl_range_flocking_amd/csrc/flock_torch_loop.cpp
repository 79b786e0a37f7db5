// flock_torch_loop.cpp — torch.classes.flock.ScTrainLoop: the config-3 training loop (BASELINE config 3, the
// reference's learners/maddpg_shared_critic/train_flock.py:112-123 cadence: env.step, store_transitions, one learn()
// per step) enqueued K steps per call from C++, so the host cost of a vectorized step is a few launch calls instead
// of a Python round trip through the step op and the learner (the per-step path: VecFlockEnv.step(ring=...) through
// flock::step_v2_store + SharedCriticLearner.pipeline_learn).
//
// Per step s (global index first + s), exactly what that per-step path enqueues:
//   env stream      flock_step_v2_ext with the fused replay insert (FlockRing rows (counter + skip) mod capacity,
//                   prev_obs = the current observation buffer), the env's double-buffered dnn / nn_idx flipped;
//   env + learner   learn() of agent (first + s) mod n_agents through the native pipeline (flock_sc_pipeline_learn:
//                   minibatch snapshot on the env stream, one merged round on the learner stream), once the ring
//                   holds a batch.
// The loop owns the pipeline (built from the learner's tensors, as SharedCriticLearner.pipeline() builds it) and the
// host mirrors of the env parity, the ring counter and the learn counter; state() returns them so the Python
// objects can be brought up to date. Results are bitwise those of the per-step path
// (tests/test_gpu_train_loop.py).
#include <ATen/ATen.h>
#include <ATen/DeviceGuard.h>
#include <hip/hip_runtime_api.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include <vector>

#include "flock_amd.h"
#include "flock_learn.h"

namespace {

using at::Tensor;

template <typename T>
T* ptr_or_null(const Tensor& t) {
    return t.defined() && t.numel() > 0 ? static_cast<T*>(t.data_ptr()) : nullptr;
}

void f32(const Tensor& t, const char* name, int64_t numel, const Tensor& like) {
    TORCH_CHECK(t.device() == like.device() && t.scalar_type() == at::kFloat && t.is_contiguous() &&
                    t.numel() == numel,
                "ScTrainLoop: ", name, " must be a contiguous f32 tensor of ", numel, " elements on ", like.device());
}

struct ScTrainLoop : torch::CustomClassHolder {
    // env: [pos, heading, vel, dnn0, dnn1, idx0, idx1, reward, done, any_done, seeds] (idx / seeds may be empty)
    std::vector<Tensor> env;
    int64_t E, N, k, launches;
    bool periodic, rigid;
    double box, sensor_range, cd, dt, v_min, v_max;
    int64_t parity;
    // replay ring of the shared critic: [state, action, reward, new_state, terminal]
    std::vector<Tensor> ring;
    int64_t capacity, counter;
    // learner
    std::vector<Tensor> keep;  // every tensor the pipeline's FlockScUpdates point into (kept alive)
    FlockScPipeline* pipe = nullptr;
    int64_t batch, n_agents, seed, learn_calls;

    ScTrainLoop(std::vector<Tensor> env_, std::vector<double> env_f, std::vector<int64_t> env_i,
                std::vector<Tensor> ring_, int64_t counter_, std::vector<Tensor> learner, std::vector<Tensor> slots,
                std::vector<int64_t> dims, std::vector<double> hyper, int64_t seed_, int64_t learn_calls_)
        : env(std::move(env_)), ring(std::move(ring_)), counter(counter_), seed(seed_), learn_calls(learn_calls_) {
        TORCH_CHECK(env.size() == 11, "ScTrainLoop: env = [pos, heading, vel, dnn0, dnn1, idx0, idx1, reward, done, "
                    "any_done, seeds]");
        TORCH_CHECK(env_f.size() == 6 && env_i.size() == 5,
                    "ScTrainLoop: env_f = [box, sensor_range, collision_distance, dt, v_min, v_max], env_i = [k, "
                    "periodic, rigid_boundary, launches, parity]");
        const Tensor& pos = env[0];
        TORCH_CHECK(pos.device().is_cuda() && pos.dim() == 3 && pos.size(2) == 2, "ScTrainLoop: pos [E, N, 2] on HIP");
        E = pos.size(0);
        N = pos.size(1);
        box = env_f[0], sensor_range = env_f[1], cd = env_f[2], dt = env_f[3], v_min = env_f[4], v_max = env_f[5];
        k = env_i[0], periodic = env_i[1] != 0, rigid = env_i[2] != 0, launches = env_i[3], parity = env_i[4] & 1;
        TORCH_CHECK(k >= 1 && k + 1 <= N, "selected index k out of range");
        TORCH_CHECK(launches >= 1 && launches <= 64, "ScTrainLoop: launches in [1, 64]");
        f32(env[0], "pos", E * N * 2, pos);
        f32(env[1], "heading", E * N, pos);
        f32(env[2], "vel", E * N * 2, pos);
        f32(env[3], "dnn0", E * N * k, pos);
        f32(env[4], "dnn1", E * N * k, pos);
        f32(env[7], "reward", E * N, pos);
        for (int i : {5, 6})
            TORCH_CHECK(env[i].numel() == 0 || (env[i].scalar_type() == at::kLong && env[i].numel() == E * N * k &&
                                                env[i].is_contiguous() && env[i].device() == pos.device()),
                        "ScTrainLoop: nn_idx buffers are [E, N, k] int64 (or empty)");
        TORCH_CHECK(env[8].scalar_type() == at::kBool && env[8].numel() == E * N && env[9].scalar_type() == at::kBool &&
                        env[9].numel() == E,
                    "ScTrainLoop: done [E, N] / any_done [E] bool");
        TORCH_CHECK(env[10].numel() == 0 || (env[10].scalar_type() == at::kShort && env[10].numel() == E * N * k),
                    "ScTrainLoop: seeds [E, N, k] int16 (or empty)");
        // ring (group 1: one row per agent, terminal = 1 - done; utils.py:47-54)
        TORCH_CHECK(ring.size() == 5 && ring[0].dim() >= 1, "ScTrainLoop: ring = [state, action, reward, new_state, "
                    "terminal]");
        capacity = ring[0].size(0);
        const int64_t w[5] = {k, 2, 1, k, 1};
        const char* rn[5] = {"ring state", "ring action", "ring reward", "ring new_state", "ring terminal"};
        for (int i = 0; i < 5; ++i) f32(ring[i], rn[i], capacity * w[i], pos);
        // learner: the pipeline's slots (SharedCriticLearner._slots[i]["job"]), as flock::sc_round takes them
        TORCH_CHECK(learner.size() == 13 && dims.size() == 7 && hyper.size() == 7 && dims[6] == 1,
                    "ScTrainLoop: learner state [13], dims [7] with do_adam, hyper [7]");
        TORCH_CHECK(slots.size() % 9 == 0 && slots.size() / 9 >= 2 && slots.size() / 9 <= 8,
                    "ScTrainLoop: 2..8 slots of 9 tensors");
        const int ns = (int)(slots.size() / 9);
        batch = dims[0];
        n_agents = learner[10].numel();
        TORCH_CHECK(dims[1] == k && dims[2] == 2, "ScTrainLoop: the learner's input is the k-wide observation");
        std::vector<FlockScUpdate> us(ns);
        std::vector<FlockScRows> staging(ns);
        for (int s = 0; s < ns; ++s) {
            const Tensor* j = &slots[9 * s];
            FlockScUpdate& u = us[s];
            u = FlockScUpdate{};
            u.B = (int)dims[0], u.in_dim = (int)dims[1], u.n_actions = (int)dims[2], u.fc1 = (int)dims[3],
            u.fc2 = (int)dims[4], u.update_rate = (int)dims[5], u.do_adam = 1;
            u.idx = static_cast<const int64_t*>(j[0].data_ptr());
            u.agent = static_cast<const int64_t*>(j[1].data_ptr());
            u.ring_state = static_cast<const float*>(j[2].data_ptr());
            u.ring_new_state = static_cast<const float*>(j[3].data_ptr());
            u.ring_action = static_cast<const float*>(j[4].data_ptr());
            u.ring_reward = static_cast<const float*>(j[5].data_ptr());
            u.ring_terminal = static_cast<const float*>(j[6].data_ptr());
            u.workspace = static_cast<float*>(j[7].data_ptr());
            u.critic_view = static_cast<float*>(j[8].data_ptr());
            u.critic = static_cast<float*>(learner[0].data_ptr());
            u.critic_grad = static_cast<float*>(learner[1].data_ptr());
            u.critic_exp_avg = static_cast<float*>(learner[2].data_ptr());
            u.critic_exp_avg_sq = static_cast<float*>(learner[3].data_ptr());
            u.critic_step = static_cast<int64_t*>(learner[4].data_ptr());
            u.actors = static_cast<float*>(learner[5].data_ptr());
            u.actors_grad = static_cast<float*>(learner[6].data_ptr());
            u.actors_exp_avg = static_cast<float*>(learner[7].data_ptr());
            u.actors_exp_avg_sq = static_cast<float*>(learner[8].data_ptr());
            u.actors_target = static_cast<float*>(learner[9].data_ptr());
            u.actor_steps = static_cast<int64_t*>(learner[10].data_ptr());
            u.actor_stride = learner[5].numel() / n_agents;
            u.losses = static_cast<float*>(learner[11].data_ptr());
            u.counters = static_cast<unsigned*>(learner[12].data_ptr());
            u.alpha = (float)hyper[0], u.beta = (float)hyper[1], u.gamma = (float)hyper[2], u.beta1 = (float)hyper[3],
            u.beta2 = (float)hyper[4], u.eps = (float)hyper[5], u.tau = (float)hyper[6];
            staging[s] = FlockScRows{const_cast<float*>(u.ring_state), const_cast<float*>(u.ring_new_state),
                                     const_cast<float*>(u.ring_action), const_cast<float*>(u.ring_reward),
                                     const_cast<float*>(u.ring_terminal)};
        }
        const FlockScRows rr{static_cast<float*>(ring[0].data_ptr()), static_cast<float*>(ring[3].data_ptr()),
                             static_cast<float*>(ring[1].data_ptr()), static_cast<float*>(ring[2].data_ptr()),
                             static_cast<float*>(ring[4].data_ptr())};
        keep = learner;
        keep.insert(keep.end(), slots.begin(), slots.end());
        pipe = flock_sc_pipeline_create(ns, us.data(), &rr, staging.data());
        TORCH_CHECK(pipe, "flock_sc_pipeline_create: ", flock_learn_last_error());
    }

    ~ScTrainLoop() override {
        if (pipe) flock_sc_pipeline_destroy(pipe);
    }

    // K vectorized steps from global step `first`; actions: a pool of [E, N, 2] f32 tensors (step s uses
    // actions[(first + s) % pool]); events: HIP event handles recorded around the env launches of the steps with
    // s % ev_every == 0 (pairs, in order; empty: none)
    void run(int64_t first, int64_t K, std::vector<Tensor> actions, int64_t env_stream, int64_t learner_stream,
             std::vector<int64_t> events, int64_t ev_every) {
        TORCH_CHECK(!actions.empty() && K >= 0, "ScTrainLoop.run: an action pool and K >= 0");
        for (const Tensor& a : actions) f32(a, "action", E * N * 2, env[0]);
        TORCH_CHECK(ev_every >= 1 && events.size() % 2 == 0, "ScTrainLoop.run: event pairs and ev_every >= 1");
        const at::OptionalDeviceGuard g(env[0].device());
        void* es = reinterpret_cast<void*>(env_stream);
        void* ls = reinterpret_cast<void*>(learner_stream);
        const int64_t n = E * N;
        size_t ev = 0;
        for (int64_t s = 0; s < K; ++s) {
            const int64_t step = first + s;
            const int64_t skip = n > capacity ? n - capacity : 0;
            FlockRing r{};
            r.state = static_cast<float*>(ring[0].data_ptr());
            r.action = static_cast<float*>(ring[1].data_ptr());
            r.reward = static_cast<float*>(ring[2].data_ptr());
            r.new_state = static_cast<float*>(ring[3].data_ptr());
            r.terminal = static_cast<float*>(ring[4].data_ptr());
            r.prev_obs = static_cast<const float*>(env[3 + parity].data_ptr());
            r.capacity = capacity;
            r.start = (counter + skip) % capacity;
            r.skip = skip;
            r.group = 1;
            const int nxt = (int)(parity ^ 1);
            FlockStepExt ext{&r, ptr_or_null<uint16_t>(env[10]), (int)launches, 0};
            const bool timed = s % ev_every == 0 && ev + 1 < events.size();
            if (timed) TORCH_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[ev]),
                                                  static_cast<hipStream_t>(es)) == hipSuccess, "hipEventRecord");
            const int rc = flock_step_v2_ext(
                es, (int)E, (int)N, (int)k, (float)box, (float)sensor_range, (float)cd, (float)dt, (float)v_min,
                (float)v_max, periodic, rigid, static_cast<float*>(env[0].data_ptr()),
                static_cast<float*>(env[1].data_ptr()), static_cast<const float*>(actions[step % actions.size()].data_ptr()),
                static_cast<float*>(env[2].data_ptr()), static_cast<float*>(env[3 + nxt].data_ptr()),
                ptr_or_null<int64_t>(env[5 + nxt]), static_cast<float*>(env[7].data_ptr()),
                static_cast<uint8_t*>(env[8].data_ptr()), static_cast<uint8_t*>(env[9].data_ptr()), &ext);
            TORCH_CHECK(rc == 0, "flock_step_v2_store: ", flock_last_error());
            if (timed) {
                TORCH_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[ev + 1]),
                                           static_cast<hipStream_t>(es)) == hipSuccess, "hipEventRecord");
                ev += 2;
            }
            parity = nxt;
            counter += n;
            if (counter >= batch) {  // SharedCriticLearner.pipeline_learn: learn() once the ring holds a batch
                ++learn_calls;
                const int64_t rows = counter < capacity ? counter : capacity;
                const int rl = flock_sc_pipeline_learn(pipe, es, ls, rows, (uint64_t)seed, (uint64_t)learn_calls,
                                                       step % n_agents);
                TORCH_CHECK(rl == 0, "flock_sc_pipeline_learn: ", flock_learn_last_error());
            }
        }
    }

    void flush(int64_t learner_stream) {
        TORCH_CHECK(flock_sc_pipeline_flush(pipe, reinterpret_cast<void*>(learner_stream)) == 0,
                    "flock_sc_pipeline_flush: ", flock_learn_last_error());
    }

    std::vector<int64_t> state() const { return {parity, counter, learn_calls}; }
};

}  // namespace

TORCH_LIBRARY_FRAGMENT(flock, m) {
    m.class_<ScTrainLoop>("ScTrainLoop")
        .def(torch::init<std::vector<Tensor>, std::vector<double>, std::vector<int64_t>, std::vector<Tensor>, int64_t,
                         std::vector<Tensor>, std::vector<Tensor>, std::vector<int64_t>, std::vector<double>, int64_t,
                         int64_t>())
        .def("run", &ScTrainLoop::run)
        .def("flush", &ScTrainLoop::flush)
        .def("state", &ScTrainLoop::state);
}
