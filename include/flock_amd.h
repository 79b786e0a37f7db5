/*
 * flock_amd.h — C ABI of the MI355X (gfx950) flocking-environment stepper (libflock_amd.so).
 *
 * Plain C: pointers, sizes and scalars only; no torch or HIP types in any signature. Every pointer is a DEVICE
 * pointer (HBM) unless stated otherwise; `stream` is a hipStream_t passed as an opaque pointer (NULL = default
 * stream). Calls enqueue kernels on `stream` and never synchronise. Return 0 on success, a negative
 * FLOCK_E* code otherwise; flock_last_error() then holds a message for the calling thread.
 *
 * Batched layout (E independent envs of N agents, k neighbours; row-major, contiguous):
 *   pos [E][N][2] f32 · heading, prev_heading [E][N] f32 · vel [E][N][2] f32 · action [E][N][2] f32
 *   action_id [E][N] i64 · noise [E][N][2] f32 · dnn [E][N][k] f32 · nn_idx [E][N][k] i64
 *   reward [E][N] f32 · done [E][N] u8 · any_done [E] u8 · obs memory [E][N][4][k] f32
 * State arrays marked (rw) are updated in place, as the reference mutates self.positions / self.headings.
 * nn_idx of the step entry points is read before it is written: on entry it may hold anything; when it holds an
 * earlier step's indices of the same envs (e.g. the previous step's output) the N >= 128 cell-list kNN uses them as
 * search seeds. The results never depend on its content (seeds that are out of range or repeated are ignored, and
 * every seeded search is exact by construction).
 *
 * Each entry point replaces one reference step()/reset() (paths relative to RetamalVictor/marl-range-flocking):
 *   flock_step_v2          environments/gym_flock_v2.py:71-83  (periodic=1; the RNN fork
 *                          learners/maddpg_official_rnn/gym_flock_v2.py:71-82 is periodic=0, v_min=0.5)
 *   flock_step_uw          environments/gym_flock_uw.py:69-81
 *   flock_step_uw_discrete environments/gym_flock_uw_discrete.py:110-122
 *   flock_step_flock       environments/gym_flock.py:48-60
 *   flock_knn              _computePeriodicDistances gym_flock_v2.py:135-151 / _computeDistances :155-175
 *   flock_reset            reset() gym_flock_v2.py:85-108, gym_flock_uw.py:83-111,
 *                          gym_flock_uw_discrete.py:124-156, gym_flock.py:62-77 (bounded in-kernel rejection
 *                          sampling instead of unbounded recursion)
 * Limits of this build: 1 <= k <= 15, k + 1 <= N <= 1024.
 */
#ifndef FLOCK_AMD_H
#define FLOCK_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FLOCK_ABI_VERSION 1

enum {
    FLOCK_OK = 0,
    FLOCK_E_K_RANGE = -1,   /* k + 1 > N ("selected index k out of range", as torch.topk raises) or k < 1 */
    FLOCK_E_LIMIT = -2,     /* outside this build's limits (k > 15 or N > 1024) */
    FLOCK_E_NULL = -3,      /* a required pointer is NULL */
    FLOCK_E_LAUNCH = -4,    /* HIP launch error */
    FLOCK_E_ARG = -5        /* other invalid argument */
};

/* variants for flock_reset */
enum { FLOCK_VARIANT_V2 = 0, FLOCK_VARIANT_UW = 1, FLOCK_VARIANT_UW_DISCRETE = 2, FLOCK_VARIANT_FLOCK = 3 };

int flock_abi_version(void);
const char* flock_last_error(void);
/* Diagnostics (A/B tests and tools only; the defaults are the product paths): "env_launches" (n launches over env
 * ranges per step), "no_spec" (generic step instantiations), "no_split" (one lane per agent in the split-scan
 * instantiations), "no_cells" (full scans instead of the cell list), "pf" (-1 default / 0 off: the env blocks' L2
 * pull-ahead of a later block's inputs in the shapes compiled with it), "sc_no_spec" (generic shared-critic row
 * kernels at fc 400/300), "sc_event_system_scope" (the learn() pipeline's events as HIP's default system-scope fences
 * instead of device-scope releases; read when a pipeline is created), "sc_free_events" (every learn() slot freed by
 * a learner-stream event, as in round 5, instead of on the device for gated single-GPU learns), "rollout_spl" (2 or 4
 * lanes per agent in the uw rollout kernel). The library reads no environment variable for them: flock_set_diag is the only way to
 * set them (process-wide; not thread-safe against concurrent launches). Returns FLOCK_OK, or FLOCK_E_ARG for an
 * unknown name. */
int flock_set_diag(const char* name, int value);

/* gym_flock_v2 step: pos (rw), heading (rw), action [lin, ang] → vel, dnn, nn_idx, reward, done, any_done. */
int flock_step_v2(void* stream, int E, int N, int k, float box, float sensor_range, float collision_distance,
                  float dt, float v_min, float v_max, int periodic, int rigid_boundary,
                  float* pos, float* heading, const float* action,
                  float* vel, float* dnn, int64_t* nn_idx, float* reward, uint8_t* done, uint8_t* any_done);

/* The same step fused with the replay insert of the training loop that drives it. Two row layouts:
 *  group = 1 (learners/maddpg_shared_critic/train_flock.py:112-127: step, then store_transitions(state, action,
 *   reward, new_state, done), utils.py:47-54): agent a = env * N + i owns ring row (start + a) mod capacity:
 *   state[k] = prev_obs[a][0..k), action[2] = the raw action, reward, new_state[k] = the new dnn row,
 *   terminal = 1 - done;
 *  group = N (main.py:41 / learners/maddpg_official_rnn/train_flock.py:45: add_record(obs["actors"],
 *   next_obs["actors"], actions, state, next_state, reward, done[0]), memory_rnn.py:53-67): env e owns ring row
 *   (start + e) mod capacity and agent i its slot i of that row: state[row][i][k], action[row][i][2],
 *   reward[row][i], new_state[row][i][k], terminal[row][i]; actor_state / actor_new_state (may be NULL) receive
 *   the same observation rows again (the record's actor copies).
 * store_done: 0 stores 1 - done (the shared critic's terminal), 1 stores done (the RNN-MADDPG record).
 * When the step produces more rows than capacity only the last `capacity` survive (as in a ring insert): units
 * (agents or envs) u < skip write nothing and unit u >= skip writes row (start + u - skip) mod capacity.
 * Requires 0 <= skip, rows - skip <= capacity and 0 <= start < capacity. */
typedef struct FlockRing {
    float* state;
    float* action;
    float* reward;
    float* new_state;
    float* terminal;
    const float* prev_obs;
    int64_t capacity;
    int64_t start;
    int64_t skip;
    float* actor_state;
    float* actor_new_state;
    int64_t group;
    int store_done;
    int action_ids; /* 1: action is the uw_discrete step's action id per agent, stored as f32 ([rows][group]) */
    int env_done;   /* 1 (group = N): terminal is one flag per env row, the env's any_done (the VDN team done) */
} FlockRing;
int flock_step_v2_store(void* stream, int E, int N, int k, float box, float sensor_range, float collision_distance,
                        float dt, float v_min, float v_max, int periodic, int rigid_boundary,
                        float* pos, float* heading, const float* action,
                        float* vel, float* dnn, int64_t* nn_idx, float* reward, uint8_t* done, uint8_t* any_done,
                        const FlockRing* ring);

/* Optional extras of the *_ext entry points (each equals its plain entry point when ext is NULL or all-NULL):
 *  ring  (v2 and uw_discrete; may be NULL): the fused replay insert of flock_step_v2_store (uw_discrete: the VDN
 *        team transition of learners/vdn/train_flock.py:102, with action_ids = 1 and env_done = 1);
 *  seeds (may be NULL): [E][N][k] u16 (rw), a compact side buffer of kNN search seeds. When set, the N >= 128
 *        cell-list kNN reads its seeds here instead of from nn_idx on entry (2 B instead of 8 B per seed) and
 *        writes this step's neighbour indices back for the next step. Any content is valid (out-of-range or repeated
 *        seeds are ignored; results never depend on it); zeroes or a reset simply fall back to a proved scan. */
typedef struct FlockStepExt {
    const FlockRing* ring;
    uint16_t* seeds;
    /* > 1: the step as that many back-to-back launches over consecutive env ranges (identical results; envs are
     * independent). While another stream's kernels run beside the step (the config-3 learner rounds), the boundary
     * between two launches lets them take the block slots the first launch's tail frees. 0 or 1: one launch. */
    int launches;
    /* != 0: normalize_distance=True of the reference constructors: the kNN (observation, collisions, rewards built
     * on them) runs on positions / max_i |p_i| of each env (gym_flock_uw.py:125-133, gym_flock_uw_discrete.py:173-181,
     * gym_flock.py:92-98, learners/maddpg_official_rnn/gym_flock_v2.py:134-141); state and centre-of-mass terms keep
     * the raw positions. Ignored by the periodic v2 step (gym_flock_v2.py:135-151 never normalises). Such steps take
     * the full-scan kernels (no cell list). */
    int normalize_distance;
} FlockStepExt;
int flock_step_v2_ext(void* stream, int E, int N, int k, float box, float sensor_range, float collision_distance,
                      float dt, float v_min, float v_max, int periodic, int rigid_boundary,
                      float* pos, float* heading, const float* action,
                      float* vel, float* dnn, int64_t* nn_idx, float* reward, uint8_t* done, uint8_t* any_done,
                      const FlockStepExt* ext);

/* gym_flock_uw step: velocity actions; obs memory mem_in → mem_out (may alias); prev_heading (rw). nn_idx may be
 * NULL (the reference does not keep it for this env). */
int flock_step_uw(void* stream, int E, int N, int k, float box, float sensor_range, float collision_distance,
                  float dt, int rigid_boundary,
                  float* pos, const float* heading, float* prev_heading, const float* action,
                  const float* mem_in, float* mem_out,
                  float* vel, float* dnn, int64_t* nn_idx, float* reward, uint8_t* done, uint8_t* any_done);

/* K gym_flock_uw steps in one call (the random-action rollout regime: the K actions are known up front; BASELINE
 * config 2 runs it): actions [K][E][N][2]; step t writes obs_out[t] ([E][N][4][k], the observation memory after the
 * step), reward_out[t] ([E][N]), done_out[t] ([E][N]) and any_done_out[t] ([E]). On return pos, vel, prev_heading,
 * mem_out, dnn, nn_idx (may be NULL), reward, done and any_done hold the state after step K - 1, exactly as K
 * flock_step_uw calls leave it (mem_in is read before anything is written: it may alias mem_out). At N = 64, k = 4
 * (config 2) one launch runs all K steps with the env state kept on chip; other shapes (and normalize_distance) run K
 * step launches. ext: seeds / launches / normalize_distance as for flock_step_uw_ext (no ring). Replaces K calls of
 * environments/gym_flock_uw.py:69-81. */
int flock_rollout_uw(void* stream, int K, int E, int N, int k, float box, float sensor_range, float collision_distance,
                     float dt, int rigid_boundary, float* pos, const float* heading, float* prev_heading,
                     const float* actions, const float* mem_in, float* mem_out, float* vel, float* dnn,
                     int64_t* nn_idx, float* reward, uint8_t* done, uint8_t* any_done, float* obs_out,
                     float* reward_out, uint8_t* done_out, uint8_t* any_done_out, const FlockStepExt* ext);

/* gym_flock_uw_discrete step: action_id indexes table [n_actions][2] (action_dictionary means). noise [E][N][2]
 * holds the N(0, noise_std) draws torch.normal adds to the means; if noise is NULL they are drawn in-kernel from
 * Philox4x32-10(seed, counter = (agent, rng_offset)). status (may be NULL): device int, bit 0 set if any action id
 * was outside [0, n_actions) (the reference raises KeyError); such agents get id 0. */
int flock_step_uw_discrete(void* stream, int E, int N, int k, float box, float sensor_range,
                           float collision_distance, float dt, float v_max, int rigid_boundary,
                           float* pos, float* heading, float* prev_heading, const int64_t* action_id,
                           const float* noise, float noise_std, uint64_t seed, uint64_t rng_offset,
                           const float* table, int n_actions,
                           float* vel, float* dnn, int64_t* nn_idx, float* reward, uint8_t* done, uint8_t* any_done,
                           int* status);

/* gym_flock (original) step: vel (rw) holds the unit velocity state; obs memory mem_in → mem_out. */
int flock_step_flock(void* stream, int E, int N, int k, float box, float collision_distance, float dt,
                     int rigid_boundary, float* pos, float* vel, const float* action,
                     const float* mem_in, float* mem_out,
                     float* dnn, int64_t* nn_idx, float* reward, uint8_t* done, uint8_t* any_done);
int flock_step_uw_ext(void* stream, int E, int N, int k, float box, float sensor_range, float collision_distance,
                      float dt, int rigid_boundary,
                      float* pos, const float* heading, float* prev_heading, const float* action,
                      const float* mem_in, float* mem_out,
                      float* vel, float* dnn, int64_t* nn_idx, float* reward, uint8_t* done, uint8_t* any_done,
                      const FlockStepExt* ext);
int flock_step_uw_discrete_ext(void* stream, int E, int N, int k, float box, float sensor_range,
                               float collision_distance, float dt, float v_max, int rigid_boundary,
                               float* pos, float* heading, float* prev_heading, const int64_t* action_id,
                               const float* noise, float noise_std, uint64_t seed, uint64_t rng_offset,
                               const float* table, int n_actions,
                               float* vel, float* dnn, int64_t* nn_idx, float* reward, uint8_t* done,
                               uint8_t* any_done, int* status, const FlockStepExt* ext);
int flock_step_flock_ext(void* stream, int E, int N, int k, float box, float collision_distance, float dt,
                         int rigid_boundary, float* pos, float* vel, const float* action,
                         const float* mem_in, float* mem_out,
                         float* dnn, int64_t* nn_idx, float* reward, uint8_t* done, uint8_t* any_done,
                         const FlockStepExt* ext);

/* Sensing only: kNN of every agent from positions (no state change). clamp != 0 clamps to [0, sensor_range]. */
int flock_knn(void* stream, int E, int N, int k, float box, float sensor_range, int periodic, int clamp,
              const float* pos, float* dnn, int64_t* nn_idx);

/*
 * Device-side reset of the envs whose env_mask[e] != 0 (env_mask may be NULL = all). Draws positions and headings
 * with the variant's distribution from Philox4x32-10(seed, counter = (agent, rng_offset + attempt)), applies
 * check_boundary, and redraws the env while any Euclidean kNN distance is below check_distance, at most
 * max_attempts times (the reference recurses without bound). Zeroes vel and prev_heading, and writes the reset
 * observation: dnn (all variants) and, when mem is non-NULL, the 4-frame memory [dnn, 0, 0, 0].
 * valid[e] (may be NULL) = 1 if the final draw is collision-free. range_lo/range_hi = range_start.
 */
int flock_reset(void* stream, int variant, int E, int N, int k, float range_lo, float range_hi, float box,
                float sensor_range, float check_distance, int rigid_boundary, int max_attempts,
                uint64_t seed, uint64_t rng_offset, const uint8_t* env_mask,
                float* pos, float* heading, float* prev_heading, float* vel, float* dnn, int64_t* nn_idx,
                float* mem, uint8_t* valid);

/* flock_reset plus a repair stage (repair_rounds > 0; flock_reset(...) == flock_reset_ext(..., 0)): an env whose
 * max_attempts whole-swarm draws all collided keeps its last draw, and every agent closer than check_distance to a
 * lower-indexed agent re-draws its own position, for up to repair_rounds rounds; the reference's kNN collision
 * check then sets valid[e]. Replaces the recursion of gym_flock_v2.py:105-108 where it cannot terminate (N >= 256
 * at main.py density: the reference overflows Python's recursion limit). */
int flock_reset_ext(void* stream, int variant, int E, int N, int k, float range_lo, float range_hi, float box,
                    float sensor_range, float check_distance, int rigid_boundary, int max_attempts,
                    uint64_t seed, uint64_t rng_offset, const uint8_t* env_mask,
                    float* pos, float* heading, float* prev_heading, float* vel, float* dnn, int64_t* nn_idx,
                    float* mem, uint8_t* valid, int repair_rounds);

/* flock_reset_ext plus normalize_distance (!= 0): the collision check and the reset observation use the kNN of
 * positions / max_i |p_i| (the reference's reset() calls _computeDistances, gym_flock_v2.py:100 / :155-163 and
 * siblings); the repair stage is off then (repair_rounds is ignored: it works on raw distances). */
int flock_reset_ext2(void* stream, int variant, int E, int N, int k, float range_lo, float range_hi, float box,
                     float sensor_range, float check_distance, int rigid_boundary, int max_attempts,
                     uint64_t seed, uint64_t rng_offset, const uint8_t* env_mask,
                     float* pos, float* heading, float* prev_heading, float* vel, float* dnn, int64_t* nn_idx,
                     float* mem, uint8_t* valid, int repair_rounds, int normalize_distance);

#ifdef __cplusplus
}
#endif

#endif /* FLOCK_AMD_H */
