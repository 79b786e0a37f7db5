// flock_torch_loop.cpp — the shared-critic learn() pipeline and the config-3 training loop as torch custom classes.
//
// torch.classes.flock.ScPipeline: the native learn() pipeline of one SharedCriticLearner (flock_sc_pipeline_*,
//   include/flock_learn.h): its staging slots, events and the pending actor phase. learn() enqueues Agent.learn() of
//   one agent (agent_simple_shared_critic.py:115-185): the minibatch snapshot on the env stream, one merged round on
//   the learner stream. ONE object per learner: the per-step Python path (SharedCriticLearner.pipeline_learn) and the
//   C++ loop below drive the same object, so the pending actor phase and the slot rotation carry over between them.
//   set_dp() turns every round into the data-parallel form (gradients into the [critic | actor] bucket, a SUM
//   all-reduce over the c10d ProcessGroup enqueued on the learner stream, the Adam launch with grad_scale = 1 / world;
//   SharedCriticLearner.dp_learn). set_rccl() makes the same collectives direct RCCL calls (ncclAllReduce on the
//   pipeline's streams over communicators of its own, one for the critic and one for the actor part) instead of
//   c10d ProcessGroup calls: the host cost of a collective drops from tens of microseconds (work objects, events,
//   stream guards) to the RCCL enqueue, which at N > 1 is what sets the step (tools/rccl_host_cost.py).
// torch.classes.flock.ScTrainLoop: the config-3 training loop (BASELINE config 3, the reference's
//   learners/maddpg_shared_critic/train_flock.py:112-123 cadence: env.step, store_transitions, one learn() per step)
//   enqueued K steps per call from C++, so the host cost of a vectorized step is a few launch calls instead of a
//   Python round trip through the step op and the learner (the per-step path: VecFlockEnv.step(ring=...) through
//   flock::step_v2_store + SharedCriticLearner.pipeline_learn).
//
// Per step s (global index first + s), exactly what that per-step path enqueues:
//   env stream      flock_step_v2_ext with the fused replay insert (FlockRing rows (counter + skip) mod capacity,
//                   prev_obs = the current observation buffer), the env's double-buffered dnn / nn_idx flipped;
//   env + learner   learn() of agent (first + s) mod n_agents through the pipeline, once the ring holds a batch.
// The loop keeps host mirrors of the env parity, the ring counter and the learn counter; set_state() loads the Python
// objects' values before a call (per-step Python steps may have run in between) and state() returns them after it.
// Results are bitwise those of the per-step path (tests/test_gpu_train_loop.py, tests/test_gpu_dist.py).
#include <ATen/ATen.h>
#include <ATen/DeviceGuard.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/custom_class.h>
#include <torch/library.h>

#include <dlfcn.h>

#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "flock_amd.h"
#include "flock_learn.h"
#include "flock_torch_sc.h"

namespace {

using at::Tensor;

// The RCCL entry points the direct path needs, resolved from the librccl torch itself loaded (librccl.so.1: one RCCL
// in the process, the one ProcessGroupNCCL uses), with the ABI types spelled out (rccl.h: ncclUniqueId is 128 bytes,
// ncclFloat32 = 7, ncclSum = 0, ncclSuccess = 0).
struct RcclUid {
    char internal[128];
};
typedef struct RcclComm* RcclCommT;
struct RcclApi {
    int (*get_unique_id)(RcclUid*) = nullptr;
    int (*comm_init_rank)(RcclCommT*, int, RcclUid, int) = nullptr;
    int (*all_reduce)(const void*, void*, size_t, int, int, RcclCommT, hipStream_t) = nullptr;
    int (*comm_destroy)(RcclCommT) = nullptr;
    const char* (*error_string)(int) = nullptr;
    bool ok = false;
};
const RcclApi& rccl() {
    static RcclApi api = [] {
        RcclApi a;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
        if (!h) return a;
        a.get_unique_id = reinterpret_cast<int (*)(RcclUid*)>(dlsym(h, "ncclGetUniqueId"));
        a.comm_init_rank = reinterpret_cast<int (*)(RcclCommT*, int, RcclUid, int)>(dlsym(h, "ncclCommInitRank"));
        a.all_reduce = reinterpret_cast<int (*)(const void*, void*, size_t, int, int, RcclCommT, hipStream_t)>(
            dlsym(h, "ncclAllReduce"));
        a.comm_destroy = reinterpret_cast<int (*)(RcclCommT)>(dlsym(h, "ncclCommDestroy"));
        a.error_string = reinterpret_cast<const char* (*)(int)>(dlsym(h, "ncclGetErrorString"));
        a.ok = a.get_unique_id && a.comm_init_rank && a.all_reduce && a.comm_destroy;
        return a;
    }();
    return api;
}
constexpr int kRcclFloat32 = 7, kRcclSum = 0;

template <typename T>
T* ptr_or_null(const Tensor& t) {
    return t.defined() && t.numel() > 0 ? static_cast<T*>(t.data_ptr()) : nullptr;
}

void f32(const Tensor& t, const char* name, int64_t numel, const Tensor& like) {
    TORCH_CHECK(t.device() == like.device() && t.scalar_type() == at::kFloat && t.is_contiguous() &&
                    t.numel() == numel,
                "ScTrainLoop: ", name, " must be a contiguous f32 tensor of ", numel, " elements on ", like.device());
}

struct ScPipeline : torch::CustomClassHolder {
    std::vector<Tensor> keep;  // every tensor the pipeline's FlockScUpdates point into (kept alive)
    FlockScPipeline* pipe = nullptr;
    at::Device device = at::Device(at::kCPU);
    int64_t batch = 0, in_dim = 0, n_actions = 0, n_agents = 0, n_slots = 0;
    // data-parallel rounds
    c10::intrusive_ptr<c10d::ProcessGroup> pg, pg_actor;
    // set_rccl: direct RCCL collectives instead of pg / pg_actor. A communicator is used from ONE stream only (two
    // collectives of one communicator on different streams could run concurrently), bound when it is made: the
    // critic part's first communicator to the learner stream set_rccl names, the second to the pipeline's comm stream
    // (split rounds' early part), the actor part's to the pipeline's actor stream. Any other stream is an error.
    RcclCommT comm_c[2] = {nullptr, nullptr};
    void* comm_c_stream[2] = {nullptr, nullptr};
    RcclCommT comm_actor = nullptr;
    void* rccl_learner_stream = nullptr;
    Tensor bucket, grad_scale;
    std::vector<Tensor> actor_grads;
    std::string cb_error;

    // learner: the 13 state tensors; slots: n_slots jobs of 9 tensors (SharedCriticLearner._slots[i]["job"]: the
    // slot's staging rows, workspace and critic view); ring: the replay ring's [state, new_state, action, reward,
    // terminal]; dims / hyper: as flock::sc_round takes them (do_adam = 1)
    ScPipeline(std::vector<Tensor> learner, std::vector<Tensor> slots, std::vector<Tensor> ring,
               std::vector<int64_t> dims, std::vector<double> hyper) {
        TORCH_CHECK(learner.size() == 13 && dims.size() == 7 && hyper.size() == 7 && dims[6] == 1,
                    "ScPipeline: learner state [13], dims [7] with do_adam = 1, hyper [7]");
        TORCH_CHECK(slots.size() % 9 == 0 && slots.size() / 9 >= 2 && slots.size() / 9 <= 8,
                    "ScPipeline: 2..8 slots of 9 tensors");
        TORCH_CHECK(ring.size() == 5, "ScPipeline: ring = [state, new_state, action, reward, terminal]");
        TORCH_CHECK(learner[0].device().is_cuda(), "ScPipeline: the learner lives on a HIP device (no CPU fallback)");
        device = learner[0].device();
        n_slots = (int64_t)(slots.size() / 9);
        batch = dims[0], in_dim = dims[1], n_actions = dims[2];
        n_agents = learner[10].numel();
        const at::TensorList L(learner);
        std::vector<FlockScUpdate> us(n_slots);
        std::vector<FlockScRows> staging(n_slots);
        for (int64_t s = 0; s < n_slots; ++s) {
            const at::TensorList job = at::TensorList(slots).slice(9 * s, 9);
            flock_torch::sc_round_checks(L, job, dims, hyper, "slot");
            TORCH_CHECK(job[8].numel() > 0, "ScPipeline: every slot needs its own critic view");
            us[s] = flock_torch::sc_update(L, job, dims, hyper);
            staging[s] = FlockScRows{static_cast<float*>(job[2].data_ptr()), static_cast<float*>(job[3].data_ptr()),
                                     static_cast<float*>(job[4].data_ptr()), static_cast<float*>(job[5].data_ptr()),
                                     static_cast<float*>(job[6].data_ptr())};
        }
        for (const Tensor& t : ring)
            TORCH_CHECK(t.device() == device && t.scalar_type() == at::kFloat && t.is_contiguous(),
                        "ScPipeline: ring fields are contiguous f32 tensors on ", device);
        const FlockScRows rr{static_cast<float*>(ring[0].data_ptr()), static_cast<float*>(ring[1].data_ptr()),
                             static_cast<float*>(ring[2].data_ptr()), static_cast<float*>(ring[3].data_ptr()),
                             static_cast<float*>(ring[4].data_ptr())};
        keep = learner;
        keep.insert(keep.end(), slots.begin(), slots.end());
        keep.insert(keep.end(), ring.begin(), ring.end());
        const at::OptionalDeviceGuard g(device);
        pipe = flock_sc_pipeline_create((int)n_slots, us.data(), &rr, staging.data());
        TORCH_CHECK(pipe, "flock_sc_pipeline_create: ", flock_learn_last_error());
    }

    ~ScPipeline() override {
        if (pipe) flock_sc_pipeline_destroy(pipe);
        for (RcclCommT c : comm_c)
            if (c) rccl().comm_destroy(c);
        if (comm_actor) rccl().comm_destroy(comm_actor);
    }

    // one RCCL unique id (128 bytes) per call, made on ONE rank and sent to the others (SharedCriticLearner.pipeline)
    static Tensor rccl_unique_id() {
        TORCH_CHECK(rccl().ok, "ScPipeline.rccl_unique_id: RCCL (librccl.so.1) is not loaded");
        RcclUid id;
        const int rc = rccl().get_unique_id(&id);
        TORCH_CHECK(rc == 0, "ncclGetUniqueId failed: ", rccl().error_string ? rccl().error_string(rc) : "");
        Tensor t = at::empty({128}, at::TensorOptions().dtype(at::kByte));
        std::memcpy(t.data_ptr(), id.internal, 128);
        return t;
    }
    static RcclCommT rccl_comm(const Tensor& uid, int64_t rank, int64_t world) {
        TORCH_CHECK(uid.device().is_cpu() && uid.scalar_type() == at::kByte && uid.numel() == 128 && uid.is_contiguous(),
                    "ScPipeline.set_rccl: the unique ids are 128-byte CPU uint8 tensors");
        RcclUid id;
        std::memcpy(id.internal, uid.data_ptr(), 128);
        RcclCommT c = nullptr;
        const int rc = rccl().comm_init_rank(&c, (int)world, id, (int)rank);
        TORCH_CHECK(rc == 0 && c, "ncclCommInitRank failed: ", rccl().error_string ? rccl().error_string(rc) : "");
        return c;
    }
    // the data-parallel collectives as direct RCCL calls (after set_dp / set_dp_actor): a communicator for the critic
    // part on learner_stream (every learn / flush / loop call of this pipeline must then use that stream), one for the
    // critic part on the pipeline's comm stream (split rounds) and one for the actor part (actor stream), every rank
    // calling with the same ids. uids: [critic (learner stream), critic (comm stream), actor], each [128] uint8 (CPU)
    void set_rccl(std::vector<Tensor> uids, int64_t rank, int64_t world, int64_t learner_stream) {
        TORCH_CHECK(rccl().ok, "ScPipeline.set_rccl: RCCL (librccl.so.1) is not loaded");
        TORCH_CHECK(pg, "ScPipeline.set_rccl: call set_dp first");
        TORCH_CHECK(uids.size() == 3, "ScPipeline.set_rccl: three unique ids");
        TORCH_CHECK(!comm_c[0], "ScPipeline.set_rccl: already set");
        TORCH_CHECK(learner_stream != 0, "ScPipeline.set_rccl: name the learner stream the rounds run on");
        const at::OptionalDeviceGuard g(device);
        rccl_learner_stream = reinterpret_cast<void*>(learner_stream);
        comm_c[0] = rccl_comm(uids[0], rank, world);
        comm_c_stream[0] = rccl_learner_stream;
        comm_c[1] = rccl_comm(uids[1], rank, world);
        comm_c_stream[1] = flock_sc_pipeline_comm_stream(pipe);  // NULL unless split: then never called
        if (pg_actor) comm_actor = rccl_comm(uids[2], rank, world);
    }
    RcclCommT critic_comm(void* stream) const {
        for (int i = 0; i < 2; ++i)
            if (comm_c_stream[i] && comm_c_stream[i] == stream) return comm_c[i];
        return nullptr;  // not a stream a communicator was bound to
    }
    void check_learner_stream(int64_t learner_stream, const char* fn) const {
        TORCH_CHECK(!rccl_learner_stream || reinterpret_cast<void*>(learner_stream) == rccl_learner_stream, fn,
                    ": the RCCL communicators are bound to the learner stream set_rccl named; enqueue the rounds there");
    }
    static int rccl_sum(RcclCommT c, float* data, int64_t n, void* stream, std::string& err) {
        const int rc = rccl().all_reduce(data, data, (size_t)n, kRcclFloat32, kRcclSum, c,
                                         static_cast<hipStream_t>(stream));
        if (rc != 0) {
            err = std::string("ncclAllReduce failed: ") + (rccl().error_string ? rccl().error_string(rc) : "");
            return -4;
        }
        return 0;
    }

    // the all-reduce between a data-parallel round's gradient and Adam launches: a SUM over the process group,
    // enqueued on the learner stream (RCCL: the collective's stream waits for the learner stream and the learner
    // stream for the collective; no host wait)
    static int allreduce_cb(void* ctx, float* data, int64_t n, void* stream) {
        auto* self = static_cast<ScPipeline*>(ctx);
        if (self->comm_c[0]) {
            RcclCommT c = self->critic_comm(stream);
            if (!c) {
                self->cb_error = "ScPipeline: the critic all-reduce was called from a stream no communicator is bound to";
                return -4;
            }
            return rccl_sum(c, data, n, stream, self->cb_error);
        }
        try {
            const c10::hip::HIPStream hs =
                c10::hip::getStreamFromExternal(static_cast<hipStream_t>(stream), self->device.index());
            const c10::hip::HIPStreamGuard guard(hs);
            std::vector<Tensor> ts{at::from_blob(data, {n}, at::TensorOptions().dtype(at::kFloat).device(self->device))};
            c10d::AllreduceOptions opts;
            opts.reduceOp = c10d::ReduceOp::SUM;
            self->pg->allreduce(ts, opts)->wait();
            return 0;
        } catch (const std::exception& e) {
            self->cb_error = e.what();
            return -4;
        }
    }

    // data-parallel rounds over pg: bucket [critic gradient | pad | actor gradient] (bucket[:critic_floats] must be the
    // learner state's critic_grad view), grad_scale [1] = 1 / world
    void set_dp(c10::intrusive_ptr<c10d::ProcessGroup> group, Tensor bucket_, int64_t critic_floats, int64_t actor_off,
                Tensor grad_scale_) {
        TORCH_CHECK(group, "ScPipeline.set_dp: a process group");
        TORCH_CHECK(bucket_.device() == device && bucket_.scalar_type() == at::kFloat && bucket_.is_contiguous(),
                    "ScPipeline.set_dp: the bucket is a contiguous f32 tensor on ", device);
        TORCH_CHECK(grad_scale_.device() == device && grad_scale_.scalar_type() == at::kFloat &&
                        grad_scale_.numel() == 1,
                    "ScPipeline.set_dp: grad_scale is one f32 on ", device);
        pg = std::move(group);
        bucket = bucket_;
        grad_scale = grad_scale_;
        const int rc = flock_sc_pipeline_set_dp(pipe, static_cast<float*>(bucket.data_ptr()), critic_floats, actor_off,
                                                bucket.numel(), static_cast<const float*>(grad_scale.data_ptr()),
                                                &ScPipeline::allreduce_cb, this);
        TORCH_CHECK(rc == 0, "flock_sc_pipeline_set_dp: ", flock_learn_last_error());
    }

    void check(int rc, const char* fn) {
        if (rc == 0) return;
        std::string msg = flock_learn_last_error();
        if (!cb_error.empty()) msg += " (" + cb_error + ")", cb_error.clear();
        TORCH_CHECK(false, fn, ": ", msg);
    }

    // learn() of `agent` on `rows` ring rows (min(counter, capacity)), the learn counter `counter` (Philox)
    void learn(int64_t rows, int64_t seed, int64_t counter, int64_t agent, int64_t env_stream, int64_t learner_stream) {
        TORCH_CHECK(agent >= 0 && agent < n_agents, "ScPipeline.learn: agent out of range");
        check_learner_stream(learner_stream, "ScPipeline.learn");
        const at::OptionalDeviceGuard g(device);
        check(flock_sc_pipeline_learn(pipe, reinterpret_cast<void*>(env_stream), reinterpret_cast<void*>(learner_stream),
                                      rows, (uint64_t)seed, (uint64_t)counter, agent),
              "flock_sc_pipeline_learn");
    }

    void flush(int64_t learner_stream) {
        check_learner_stream(learner_stream, "ScPipeline.flush");
        const at::OptionalDeviceGuard g(device);
        check(flock_sc_pipeline_flush(pipe, reinterpret_cast<void*>(learner_stream)), "flock_sc_pipeline_flush");
    }

    // raises if a round gave up waiting for its snapshot (device-side gate timeout; its results are invalid).
    // Synchronous: call once the learner stream has been synchronised
    void verify() {
        const at::OptionalDeviceGuard g(device);
        check(flock_sc_pipeline_check(pipe), "flock_sc_pipeline_check");
    }

    int64_t gated() const { return flock_sc_pipeline_gated(pipe); }
    int64_t gated_learns() const { return flock_sc_pipeline_gated_learns(pipe); }

    // the device gate's guard (flock_sc_pipeline_mark): wait = true records an event behind everything env_stream holds
    // now, which the next learn's round waits for on the learner stream; wait = false declares that only the caller's
    // own env step will be enqueued on env_stream before the next learn (the C++ loop after its first step). A learn
    // with no mark since the previous one takes the event hand-off (never spins behind work of unknown length)
    void mark(int64_t env_stream, bool wait) {
        const at::OptionalDeviceGuard g(device);
        check(flock_sc_pipeline_mark(pipe, reinterpret_cast<void*>(env_stream), wait ? 1 : 0), "flock_sc_pipeline_mark");
    }

    // The learner stream of a device's pipelines, created once per (device, priority) and never destroyed, so that
    // every learner of a process runs on the same stream whatever torch's stream pool holds (a pool stream can share
    // its hardware queue with the env stream once a process has more streams than GPU_MAX_HW_QUEUES: the same loop
    // then serialises, profiles/r05/rccl_host/host_cost_q4.txt). Non-blocking; high = the device's greatest priority,
    // whose streams HIP places on hardware queues apart from the normal-priority ones (the env stream's)
    static int64_t stream(int64_t device_index, bool high) { return owned_stream(device_index, high ? 1 : 0); }
    // the overlapped-train update stream of the config-4 / 5 learners (learners/core.py OverlappedTrain): normal
    // priority, distinct from the learn() pipelines' streams
    static int64_t side_stream(int64_t device_index) { return owned_stream(device_index, 2); }
    // kind 0: normal priority, 1: high priority, 2: the side stream; created once per device and kept for the process
    static int64_t owned_stream(int64_t device_index, int kind) {
        static std::mutex m;
        static std::map<std::pair<int64_t, int>, hipStream_t> streams;
        const std::lock_guard<std::mutex> lock(m);
        const auto key = std::make_pair(device_index, kind);
        auto it = streams.find(key);
        if (it != streams.end()) return reinterpret_cast<int64_t>(it->second);
        const c10::hip::HIPGuard g((c10::DeviceIndex)device_index);
        int least = 0, greatest = 0;
        TORCH_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess,
                    "ScPipeline.stream: hipDeviceGetStreamPriorityRange");
        hipStream_t s = nullptr;
        TORCH_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, kind == 1 ? greatest : least) == hipSuccess &&
                        s,
                    "ScPipeline.stream: hipStreamCreateWithPriority");
        streams[key] = s;
        return reinterpret_cast<int64_t>(s);
    }

    // the snapshot hand-off: 1 the device-side gate (the default on one GPU), 0 cross-queue event waits; returns the
    // hand-off in use (single-GPU and data-parallel pipelines alike; rocprofv3 counter collection always takes the
    // events). A learn takes the gate only after a mark (see mark below)
    int64_t set_gate(bool on) {
        const at::OptionalDeviceGuard g(device);
        return flock_sc_pipeline_set_gate(pipe, on ? 1 : 0);
    }

    // the actor half of each data-parallel round off the learner chain (flock_sc_pipeline_set_dp_actor): one actor
    // gradient buffer per slot, all-reduced (SUM) over `group` on the pipeline's actor stream
    static int actor_allreduce_cb(void* ctx, float* data, int64_t n, void* stream) {
        auto* self = static_cast<ScPipeline*>(ctx);
        if (self->comm_actor) return rccl_sum(self->comm_actor, data, n, stream, self->cb_error);
        try {
            const c10::hip::HIPStream hs =
                c10::hip::getStreamFromExternal(static_cast<hipStream_t>(stream), self->device.index());
            const c10::hip::HIPStreamGuard guard(hs);
            std::vector<Tensor> ts{at::from_blob(data, {n}, at::TensorOptions().dtype(at::kFloat).device(self->device))};
            c10d::AllreduceOptions opts;
            opts.reduceOp = c10d::ReduceOp::SUM;
            self->pg_actor->allreduce(ts, opts)->wait();
            return 0;
        } catch (const std::exception& e) {
            self->cb_error = e.what();
            return -4;
        }
    }
    void set_dp_actor(c10::intrusive_ptr<c10d::ProcessGroup> group, std::vector<Tensor> grads) {
        TORCH_CHECK(group, "ScPipeline.set_dp_actor: a process group");
        TORCH_CHECK((int64_t)grads.size() == n_slots, "ScPipeline.set_dp_actor: one actor gradient buffer per slot");
        std::vector<float*> ptrs;
        for (const Tensor& t : grads) {
            TORCH_CHECK(t.device() == device && t.scalar_type() == at::kFloat && t.is_contiguous(),
                        "ScPipeline.set_dp_actor: contiguous f32 buffers on ", device);
            ptrs.push_back(static_cast<float*>(t.data_ptr()));
        }
        pg_actor = std::move(group);
        actor_grads = grads;
        const at::OptionalDeviceGuard g(device);
        const int rc = flock_sc_pipeline_set_dp_actor(pipe, ptrs.data(), (int)n_agents, &ScPipeline::actor_allreduce_cb,
                                                      this);
        TORCH_CHECK(rc == 0, "flock_sc_pipeline_set_dp_actor: ", flock_learn_last_error());
    }
};

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
    c10::intrusive_ptr<ScPipeline> pipe;
    int64_t seed, learn_calls;
    ScTrainLoop(std::vector<Tensor> env_, std::vector<double> env_f, std::vector<int64_t> env_i,
                std::vector<Tensor> ring_, int64_t counter_, c10::intrusive_ptr<ScPipeline> pipe_, int64_t seed_,
                int64_t learn_calls_)
        : env(std::move(env_)), ring(std::move(ring_)), counter(counter_), pipe(std::move(pipe_)), seed(seed_),
          learn_calls(learn_calls_) {
        TORCH_CHECK(env.size() == 11, "ScTrainLoop: env = [pos, heading, vel, dnn0, dnn1, idx0, idx1, reward, done, "
                    "any_done, seeds]");
        TORCH_CHECK(env_f.size() == 6 && env_i.size() == 5,
                    "ScTrainLoop: env_f = [box, sensor_range, collision_distance, dt, v_min, v_max], env_i = [k, "
                    "periodic, rigid_boundary, launches, parity]");
        TORCH_CHECK(pipe, "ScTrainLoop: a learn() pipeline (torch.classes.flock.ScPipeline)");
        const Tensor& pos = env[0];
        TORCH_CHECK(pos.device().is_cuda() && pos.dim() == 3 && pos.size(2) == 2, "ScTrainLoop: pos [E, N, 2] on HIP");
        TORCH_CHECK(pos.device() == pipe->device, "ScTrainLoop: the env and the learner must share a device");
        E = pos.size(0);
        N = pos.size(1);
        box = env_f[0], sensor_range = env_f[1], cd = env_f[2], dt = env_f[3], v_min = env_f[4], v_max = env_f[5];
        k = env_i[0], periodic = env_i[1] != 0, rigid = env_i[2] != 0, launches = env_i[3], parity = env_i[4] & 1;
        TORCH_CHECK(k >= 1 && k + 1 <= N, "selected index k out of range");
        TORCH_CHECK(launches >= 1 && launches <= 64, "ScTrainLoop: launches in [1, 64]");
        TORCH_CHECK(pipe->in_dim == k && pipe->n_actions == 2, "ScTrainLoop: the learner's input is the k-wide "
                    "observation and its action the 2 controls");
        TORCH_CHECK(pipe->n_agents == N, "ScTrainLoop: one actor per agent");
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
    }

    // the Python objects' current values (VecFlockEnv._cur, ReplayRing.counter, SharedCriticLearner._learn_calls):
    // per-step Python steps may have advanced them since the last call
    void set_state(int64_t parity_, int64_t counter_, int64_t learn_calls_) {
        TORCH_CHECK(counter_ >= 0 && learn_calls_ >= 0, "ScTrainLoop.set_state: counters are >= 0");
        parity = parity_ & 1;
        counter = counter_;
        learn_calls = learn_calls_;
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
        const int64_t n = E * N;
        size_t ev = 0;
        bool marked = false;
        for (int64_t s = 0; s < K; ++s) {
            const int64_t step = first + s;
            const int64_t skip = n > capacity ? n - capacity : 0;
            const Tensor* rf = ring.data();
            FlockRing r{};
            r.state = static_cast<float*>(rf[0].data_ptr());
            r.action = static_cast<float*>(rf[1].data_ptr());
            r.reward = static_cast<float*>(rf[2].data_ptr());
            r.new_state = static_cast<float*>(rf[3].data_ptr());
            r.terminal = static_cast<float*>(rf[4].data_ptr());
            r.prev_obs = static_cast<const float*>(env[3 + parity].data_ptr());
            r.capacity = capacity;
            r.start = (counter + skip) % capacity;
            r.skip = skip;
            r.group = 1;
            const int nxt = (int)(parity ^ 1);
            FlockStepExt ext{&r, ptr_or_null<uint16_t>(env[10]), (int)launches, 0};
            // the device gate's guard, for the steps that learn: the first such step's mark waits for whatever the env
            // stream held before it; later steps declare that only this loop's own env step precedes their snapshot
            if (counter + n >= pipe->batch) {
                pipe->mark(env_stream, !marked);
                marked = true;
            }
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
            if (counter >= pipe->batch) {  // SharedCriticLearner.pipeline_learn: learn() once the ring holds a batch
                ++learn_calls;
                const int64_t rows = counter < capacity ? counter : capacity;
                pipe->learn(rows, seed, learn_calls, step % pipe->n_agents, env_stream, learner_stream);
            }
        }
    }

    void flush(int64_t learner_stream) { pipe->flush(learner_stream); }

    // [env parity, ring counter, learn() calls]
    std::vector<int64_t> state() const { return {parity, counter, learn_calls}; }
};

}  // namespace

TORCH_LIBRARY_FRAGMENT(flock, m) {
    m.class_<ScPipeline>("ScPipeline")
        .def(torch::init<std::vector<Tensor>, std::vector<Tensor>, std::vector<Tensor>, std::vector<int64_t>,
                         std::vector<double>>())
        .def("set_dp", &ScPipeline::set_dp)
        .def("learn", &ScPipeline::learn)
        .def("flush", &ScPipeline::flush)
        .def("verify", &ScPipeline::verify)
        .def("gated", &ScPipeline::gated)
        .def("gated_learns", &ScPipeline::gated_learns)
        .def("set_gate", &ScPipeline::set_gate)
        .def("mark", &ScPipeline::mark)
        .def_static("stream", &ScPipeline::stream)
        .def_static("side_stream", &ScPipeline::side_stream)
        .def("set_dp_actor", &ScPipeline::set_dp_actor)
        .def("set_rccl", &ScPipeline::set_rccl)
        .def_static("rccl_unique_id", &ScPipeline::rccl_unique_id);
    m.class_<ScTrainLoop>("ScTrainLoop")
        .def(torch::init<std::vector<Tensor>, std::vector<double>, std::vector<int64_t>, std::vector<Tensor>, int64_t,
                         c10::intrusive_ptr<ScPipeline>, int64_t, int64_t>())
        .def("set_state", &ScTrainLoop::set_state)
        .def("run", &ScTrainLoop::run)
        .def("flush", &ScTrainLoop::flush)
        .def("state", &ScTrainLoop::state);
}
