/*
 * flock_learn.h — C ABI of the learner-side HIP kernels in libflock_amd.so (gfx950).
 *
 * Device pointers, sizes, scalars; `stream` is a hipStream_t passed as an opaque pointer. Return 0 or a negative
 * code (flock_learn_last_error() holds the message). They replace, for ALL agents of a learner at once:
 *   flock_adam_step    torch.optim.Adam.step() per agent network (learners/maddpg_official_rnn/agent.py:32-33,
 *                      maddpg_shared_critic/ddpg_network.py:53,127, vdn/train_flock.py:265) fused with the
 *                      target soft update (maddpg_official_rnn/net.py:305-309 mode 0,
 *                      maddpg_shared_critic/agent_simple_shared_critic.py:158-185 mode 1)
 *   flock_soft_update  the soft update alone (same two forms)
 *   flock_grad_norm    torch.nn.utils.clip_grad_norm_ (vdn/train_flock.py:42): out[0] = ||g||_2,
 *                      out[1] = min(max_norm / (||g|| + 1e-6), 1); pass out+1 as flock_adam_step's grad_scale
 *   flock_gru_fwd/bwd  nn.GRUCell elementwise part (maddpg_official_rnn/net.py:33,118, vdn/net.py:24)
 *   flock_gather_rows  replay minibatch / chunk gather (maddpg_official_rnn/memory_rnn.py:69-99,
 *                      vdn/utils.py:31-60, maddpg_shared_critic/utils.py:65-76)
 *   flock_scatter_rows replay insertion (memory_rnn.py:53-67, maddpg_shared_critic/utils.py:47-54)
 */
#ifndef FLOCK_LEARN_H
#define FLOCK_LEARN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* flock_learn_last_error(void);

/* One Adam step over n contiguous floats (step = the optimizer's step count after incrementing, >= 1).
 * grad_scale (device float, may be NULL) multiplies the gradient first (clip_grad_norm_ coefficient).
 * target (may be NULL): soft update after the step, mode 0 t*(1-tau)+p*tau, mode 1 tau*p+(1-tau)*t. */
int flock_adam_step(void* stream, int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                    const float* grad_scale, float lr, float beta1, float beta2, float eps, int64_t step,
                    float* target, float tau, int target_mode);

/* Same, with the step count read from device memory (*step, already incremented): HIP-graph capturable. */
int flock_adam_step_dev(void* stream, int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                        const float* grad_scale, float lr, float beta1, float beta2, float eps, const int64_t* step,
                        float* target, float tau, int target_mode);

int flock_soft_update(void* stream, int64_t n, float* target, const float* src, float tau, int mode);

/* partial: device scratch of max_parts doubles; out: device float[2] */
int flock_grad_norm(void* stream, int64_t n, const float* grad, double* partial, int max_parts, float max_norm,
                    float* out);

/* rows = batch rows (all agents); gi, gh: [rows][3H]; h, hout: [rows][H]; ws: [rows][4H] (may be NULL in fwd). */
int flock_gru_fwd(void* stream, int64_t rows, int H, const float* gi, const float* gh, const float* h, float* hout,
                  float* ws);
int flock_gru_bwd(void* stream, int64_t rows, int H, const float* dhout, const float* h, const float* ws, float* dgi,
                  float* dgh, float* dh);

/* GRUCell recurrence of A networks over a whole chunk of C steps in one launch (one block per network; replaces the
 * per-step GRUCell calls of vdn/train_flock.py:23-36 and maddpg_official_rnn/MADDPG.py:95-132). gi: [A][C][B][3H]
 * input-side pre-activations x W_ih^T + b_ih of every step; w_hh [A][3H][H], b_hh [A][3H]; keep: uint8 mask at
 * keep[t*keep_st + a*keep_sa + b*keep_sb] (0: the hidden state is reset to zero after step t, the done reset);
 * initial hidden state zero. Out: hs [A][C][B][H] (each step's output before its reset), ws [A][C][B][4H] (saved
 * gates for the backward; may be NULL). H = 32; B <= 256.
 * bwd: dhs = dLoss/dhs -> dgi [A][C][B][3H], dw_hh [A][3H][H], db_hh [A][3H] (written, not accumulated). */
int flock_gru_seq_fwd(void* stream, int A, int C, int B, int H, const float* gi, const float* w_hh, const float* b_hh,
                      const uint8_t* keep, int64_t keep_st, int64_t keep_sa, int64_t keep_sb, float* hs, float* ws);
int flock_gru_seq_bwd(void* stream, int A, int C, int B, int H, const float* dhs, const float* hs, const float* ws,
                      const float* w_hh, const uint8_t* keep, int64_t keep_st, int64_t keep_sa, int64_t keep_sb,
                      float* dgi, float* dw_hh, float* db_hh);
/* The same recurrence with VDN's q head fused (learners/vdn/net.py:34-37, QNet.q = Linear(32, n_actions) on every
 * step's GRU output): q_fwd also writes q [A][C][B][NA] = hs W_q^T + b_q (w_q [A][NA][H], b_q [A][NA], NA <= 16);
 * hs and ws may be NULL together (no backward). q_bwd takes dq = dLoss/dq [A][C][B][NA] in place of dhs and also
 * writes dw_q [A][NA][H], db_q [A][NA]. Replaces the q head's batched GEMMs (forward, both backward GEMMs and the
 * bias sum) of vdn/train_flock.py:23-28's q(s) for every agent and step. */
int flock_gru_seq_q_fwd(void* stream, int A, int C, int B, int H, int NA, const float* gi, const float* w_hh,
                        const float* b_hh, const float* w_q, const float* b_q, const uint8_t* keep, int64_t keep_st,
                        int64_t keep_sa, int64_t keep_sb, float* hs, float* ws, float* q);
int flock_gru_seq_q_bwd(void* stream, int A, int C, int B, int H, int NA, const float* dq, const float* hs,
                        const float* ws, const float* w_hh, const float* w_q, const uint8_t* keep, int64_t keep_st,
                        int64_t keep_sa, int64_t keep_sb, float* dgi, float* dw_hh, float* db_hh, float* dw_q,
                        float* db_q);

/* VDN QNet feature chain of A agents, R rows each (learners/vdn/net.py:19-33; replaces the three per-agent Linear
 * layers and two ReLUs before the GRUCell, train_flock.py:23-27 runs them per chunk step):
 *   y1 = relu(x w1^T + b1) [64], y2 = relu(y1 w2^T + b2) [32], gi = y2 w_ih^T + b_ih [96]
 * x element (a, c, b, f) at x[a*x_sa + c*x_sc + b*x_sb + f] with row r = c*B + b (R = C*B); w1 [A][64][n_in],
 * b1 [A][64], w2 [A][32][64], b2 [A][32], w_ih [A][96][32], b_ih [A][96] contiguous. Out: gi [A][R][96];
 * y1 [A][R][64] and y2 [A][R][32] (the post-ReLU activations the backward needs; each may be NULL). 1 <= n_in <= 16. */
int flock_vdn_feat_fwd(void* stream, int A, int R, int B, int n_in, const float* x, int64_t x_sa, int64_t x_sc,
                       int64_t x_sb, const float* w1, const float* b1, const float* w2, const float* b2,
                       const float* w_ih, const float* b_ih, float* y1, float* y2, float* gi);

/* Backward of flock_vdn_feat_fwd (the autograd chain of vdn/train_flock.py:40 through the feature layers), one
 * launch for all agents: dgi [A][R][96] = dLoss/dgi, y1 [A][R][64] / y2 [A][R][32] the forward's post-ReLU outputs,
 * x / w2 [A][32][64] / w_ih [A][96][32] as in the forward. Writes (not accumulates) dw1 [A][64][n_in], db1 [A][64],
 * dw2 [A][32][64], db2 [A][32], dw_ih [A][96][32], db_ih [A][96]. */
int flock_vdn_feat_bwd(void* stream, int A, int R, int B, int n_in, const float* x, int64_t x_sa, int64_t x_sc,
                       int64_t x_sb, const float* w2, const float* w_ih, const float* y1, const float* y2,
                       const float* dgi, float* dw1, float* db1, float* dw2, float* db2, float* dw_ih, float* db_ih);

/* gather: dst[r][:] = src[idx[r]][:]; scatter: dst[idx[r]][:] = src[r][:]; rows of `width` floats. */
int flock_gather_rows(void* stream, int64_t rows, int64_t width, const float* src, const int64_t* idx, float* dst);
int flock_scatter_rows(void* stream, int64_t rows, int64_t width, const float* src, const int64_t* idx, float* dst);

/* Replay insert of n rows into ring rows start .. start+n-1 (mod capacity), every field in ONE launch (replaces the
 * per-field row copies of ReplayBuffer.store_transitions, maddpg_shared_critic/utils.py:47-54, memory_rnn.py:53-67,
 * vdn/utils.py:20-29). src: n * width contiguous values; dst: the field's [capacity][width] f32 ring.
 * kind 0: f32 copy; 1: u8/bool -> 1 - x (the stored "terminal"); 2: u8/bool -> x; 3: int64 -> f32 (round to
 * nearest, as torch's .float(): discrete action ids). At most 8 fields; n <= capacity. */
typedef struct FlockRingField {
    const void* src;
    float* dst;
    int64_t width;
    int kind;
} FlockRingField;
int flock_ring_store(void* stream, int64_t n, int64_t capacity, int64_t start, int nfields,
                     const FlockRingField* fields);

/* ---- fused shared-critic DDPG update ------------------------------------------------------------------------
 * Replaces Agent.learn() of learners/maddpg_shared_critic/agent_simple_shared_critic.py:115-150 (the sample,
 * target, critic MSE backward + Adam, actor -mean Q backward + Adam) for agent *agent, on the networks of
 * learners/maddpg_shared_critic/ddpg_network.py:58-70 (critic) and :132-141 (actor). The soft updates
 * (:152-185) stay separate (flock_soft_update). Parameter buffers are flat f32 in the reference's state_dict order:
 *   critic: fc1.weight [fc1,in] fc1.bias bn1.weight bn1.bias fc2.weight [fc2,fc1] fc2.bias bn2.weight bn2.bias
 *           action_value.weight [fc2,na] action_value.bias q.weight [1,fc2] q.bias [1]
 *   actor:  fc1.weight fc1.bias bn1.weight bn1.bias fc2.weight fc2.bias bn2.weight bn2.bias mu.weight [na,fc2]
 *           mu.bias [na]; agent a's actor at actors + a * actor_stride (same for grad / moments / target).
 * Replay rows are read straight from the ring (rows idx[0..B)). workspace: flock_sc_workspace_floats() floats;
 * counters: 2 zero-initialised uints (kept zero between calls). do_adam = 0 writes the gradients only (data-parallel
 * callers all-reduce them and run flock_adam_step_dev themselves); step counters are incremented only with do_adam.
 * Limits: in_dim <= 64, n_actions <= 8, fc1, fc2 <= 1024. losses[0] = actor loss, losses[1] = critic loss. */
typedef struct FlockScUpdate {
    int B, in_dim, n_actions, fc1, fc2, do_adam;
    const int64_t* idx;   /* [B] replay rows */
    const int64_t* agent; /* device scalar: the learning agent */
    const float *ring_state, *ring_new_state, *ring_action, *ring_reward, *ring_terminal;
    float *critic, *critic_grad, *critic_exp_avg, *critic_exp_avg_sq;
    int64_t* critic_step;
    float *actors, *actors_grad, *actors_exp_avg, *actors_exp_avg_sq, *actors_target;
    int64_t* actor_steps; /* [n_agents] */
    int64_t actor_stride;
    float* losses;
    float* workspace;
    unsigned* counters;
    float alpha, beta, gamma, beta1, beta2, eps;
    float tau;       /* soft-update rate (update_network_parameters, :158-185) */
    int update_rate; /* > 0 (with do_adam): flock_sc_actor_update also applies the soft updates when this agent's
                        learn count (= actor_steps[agent] before the step) is a multiple of it, after both Adam
                        steps, as Agent.learn() does (:152-154); 0: the caller runs them (flock_soft_update) */
    float* critic_view; /* may be NULL. With do_adam: flock_sc_critic_update writes the critic's post-Adam
                           parameters here and, when this learn() soft-updates (update_rate above), the critic's
                           self soft update tau c + (1 - tau) c (the shared critic is its own target, :172-178)
                           straight into `critic`. flock_sc_actor_update reads the critic from critic_view whenever
                           it is given (with do_adam = 0 too: data-parallel gradient rounds).
                           Results are bitwise those of critic_view = NULL; what it buys is that the critic phase of
                           the NEXT learn() (which reads `critic`) may run while this actor phase still reads the
                           critic it was given (two views, alternated by the caller). */
    float* actor_grad_out; /* may be NULL. The actor phase writes its gradient here (one actor, not agent-relative)
                              instead of actors_grad + agent * actor_stride, and flock_sc_round_adam reads it
                              there: data-parallel callers put it right behind critic_grad, so the two gradients
                              of a round are ONE contiguous all-reduce bucket. */
} FlockScUpdate;

int64_t flock_sc_workspace_floats(int B, int in_dim, int n_actions, int fc1, int fc2);
int64_t flock_sc_update_size(void); /* sizeof(FlockScUpdate), for binding checks */
/* learn() prologue in ONE launch: *agent_out = agent; idx[r] = Philox4x32-10(seed, counter, r) mod rows for
 * r < B (uniform sampling with replacement, ReplayBuffer.sample_buffer, utils.py:65-76). idx may be NULL. */
int flock_sc_prep(void* stream, int B, int64_t rows, uint64_t seed, uint64_t counter, int64_t* idx,
                  int64_t* agent_out, int64_t agent);
/* The same prologue with a minibatch snapshot: staging row r (r < B) receives every field of replay row
 * Philox4x32-10(seed, counter, r) mod rows (the row flock_sc_prep samples; written to idx_out when non-NULL).
 * An update whose ring pointers are the staging fields and whose idx is 0..B-1 computes exactly the update on
 * the sampled ring rows, and no longer reads the ring: the next env step may rewrite it concurrently. */
typedef struct FlockScRows {
    float* state;      /* [rows][in_dim] */
    float* new_state;  /* [rows][in_dim] */
    float* action;     /* [rows][n_actions] */
    float* reward;     /* [rows] */
    float* terminal;   /* [rows] (1 - done) */
} FlockScRows;
int flock_sc_prep_snapshot(void* stream, int B, int64_t rows, uint64_t seed, uint64_t counter, int64_t* idx_out,
                           int64_t* agent_out, int64_t agent, int in_dim, int n_actions, const FlockScRows* ring,
                           const FlockScRows* staging);
/* Agent.choose_action of every agent on every env row in one launch (learners/maddpg_shared_critic/
 * agent_simple_shared_critic.py:92-107; actor ddpg_network.py:132-141; OUActionNoiseGPU utils.py:15-18 with one
 * process per (row, agent)). obs [rows][n_agents][in_dim] f32; actors: the agent-major actor buffer of
 * FlockScUpdate (agent a at actors + a * actor_stride; 16-B aligned, actor_stride a multiple of 4); actions
 * [rows][n_agents][2] = tanh(mu head) (+ the OU state after its step when ou_state is not NULL: ou <- ou +
 * theta (0 - ou) dt + sigma_sqrt_dt noise, in that float op order, noise [rows][n_agents][2] N(0,1) draws).
 * Limits: 1 <= in_dim <= 16, fc1 a multiple of 8 (<= 2000 at in_dim 4), fc2 <= 320, 2 actions. */
int flock_sc_act(void* stream, int64_t rows, int n_agents, int in_dim, int fc1, int fc2, const float* obs,
                 const float* actors, int64_t actor_stride, float* actions, float* ou_state, const float* noise,
                 float theta, float dt, float sigma_sqrt_dt);
int flock_sc_critic_update(void* stream, const FlockScUpdate* u); /* :118-141 */
int flock_sc_actor_update(void* stream, const FlockScUpdate* u);  /* :144-150 (after the critic update) */
/* One round of six launches: the critic phase of critic_u and the actor phase of actor_u (either may be NULL; each
 * alone is flock_sc_critic_update / flock_sc_actor_update). For two learn() calls of DIFFERENT agents, round(critic
 * of call t+1, actor of call t) is bitwise the actor phase of t followed by the critic phase of t+1: the phases share
 * no written state (actor_u must carry a critic_view, critic_u its own workspace and critic_view). The two updates
 * must have the same shapes. */
int flock_sc_round(void* stream, const FlockScUpdate* critic_u, const FlockScUpdate* actor_u);
/* The Adam half of a data-parallel round: after flock_sc_round with do_adam = 0 wrote the gradients and the caller
 * all-reduced them (sums), one launch applies Adam to the whole critic (critic_u: with its critic_view and self
 * soft update, as flock_sc_critic_update with do_adam) and / or to the actor of actor_u's agent (from
 * actor_grad_out when set; its target soft update on soft learns), every gradient multiplied by *grad_scale
 * (device scalar, e.g. 1 / world; NULL: 1) first; step counters advance as with do_adam. critic_u / actor_u must
 * have do_adam = 1. */
int flock_sc_round_adam(void* stream, const FlockScUpdate* critic_u, const FlockScUpdate* actor_u,
                        const float* grad_scale);

/* learn() pipeline of a training loop that calls Agent.learn() once per env step (train_flock.py:120-121, one agent
 * per call; replaces agent_simple_shared_critic.py:115-185 called in that cadence): n_slots (2..8) staging slots, each
 * with its own FlockScUpdate (do_adam, own critic_view, own workspace; ring fields = that slot's staging rows, idx =
 * 0..B-1). flock_sc_pipeline_learn enqueues learn() t of `agent` with no host synchronisation:
 *   env_stream:     [wait until the slot's previous learn() has consumed its staging rows] minibatch snapshot
 *                   (rows sampled with Philox(seed, counter), as flock_sc_prep_snapshot)
 *   learner_stream: ONE round (five launches): the critic phase of learn t with the actor phase of learn t-1 (if
 *                   learn t-1 had the same agent: its actor phase, then this critic phase)
 * The round's wait for the snapshot is, by default, the device-side gate: the snapshot (one workgroup) stores the
 * staging rows and the agent index write-through (`sc1`), waits for its stores and publishes a sequence number; the
 * critic phase's row blocks poll it and read the staging rows `sc1` (MI355X_MICROARCH.md hand-off table, row 1). A
 * learn() is gated only when the caller called flock_sc_pipeline_mark since the previous learn():
 * mark(p, env_stream, 1) records an event behind everything env_stream holds at that point, and the round first waits
 * for it on the learner stream (a cross-queue wait that occupies no CU and is usually complete already), so the row
 * blocks spin only over the env work enqueued after the mark (the caller's own env step); mark(p, env_stream, 0)
 * declares that nothing but the caller's own env step was enqueued on env_stream since the previous learn's
 * snapshot (the C++ training loop, after its first step). Without a mark the learn() takes the cross-queue event
 * hand-off, so a learn never fails because env_stream is busy with other work. The spin stays bounded (2 s, far
 * above any env step; a waiter that gives up sets an error word and computes nothing, flock_sc_pipeline_check
 * returns -6). flock_sc_pipeline_set_gate(p, 0) (and always under rocprofv3 counter collection, which serialises
 * dispatches) makes every learn() take the event wait; it returns the hand-off in use (1 gate, 0 events). The gate
 * serves single-GPU and data-parallel pipelines alike. Slot reuse: when a learn() and the slot's previous learn() are
 * both gated, the previous round's fc2 GEMM launch (after its row launch, the staging rows' only reader; the later
 * launches carry the agent index by value) stores that learn's sequence number write-through and the new snapshot
 * polls it before writing (bounded like the gate; 60 s for data-parallel rounds, whose GEMM may sit behind an
 * all-reduce waiting for other ranks); otherwise (event hand-off, split data-parallel rounds, flock_set_diag
 * "sc_free_events") the env stream waits for a learner-stream event recorded after the round that freed the slot. Both hand-offs are deadlock-free whatever
 * hardware queues the streams map to: every snapshot is enqueued before the round that waits for it, and a snapshot
 * waits only for a round enqueued before it whose own snapshot precedes it on env_stream. The actor phase of the last learn() stays pending until the
 * next call or flock_sc_pipeline_flush (which enqueues it on learner_stream). Results are bitwise those of the serial
 * learn() sequence. Returns NULL (create) or a negative code; flock_learn_last_error() has the message. */
typedef struct FlockScPipeline FlockScPipeline;
FlockScPipeline* flock_sc_pipeline_create(int n_slots, const FlockScUpdate* slots, const FlockScRows* ring,
                                          const FlockScRows* staging);
int flock_sc_pipeline_learn(FlockScPipeline* p, void* env_stream, void* learner_stream, int64_t rows, uint64_t seed,
                            uint64_t counter, int64_t agent);
int flock_sc_pipeline_set_gate(FlockScPipeline* p, int on);
int flock_sc_pipeline_mark(FlockScPipeline* p, void* env_stream, int wait);
int flock_sc_pipeline_gated(const FlockScPipeline* p);
int64_t flock_sc_pipeline_gated_learns(const FlockScPipeline* p); /* learns so far that took the gate */
int flock_sc_pipeline_check(FlockScPipeline* p);
int flock_sc_pipeline_flush(FlockScPipeline* p, void* learner_stream);
void flock_sc_pipeline_destroy(FlockScPipeline* p);
/* Data-parallel rounds (one replica per GPU, the same learn() sequence on every rank): after this call every round
 * of the pipeline runs as gradients only (do_adam = 0, critic_grad = bucket, actor_grad_out = bucket + actor_off),
 * then `allreduce(ctx, bucket + lo, hi - lo, learner_stream)` over the part the round wrote (the critic gradient
 * [0, critic_floats) with a critic phase, the actor gradient [actor_off, bucket_floats) with an actor phase), which
 * must enqueue a SUM all-reduce of those floats on learner_stream (e.g. RCCL) and return 0, then
 * flock_sc_round_adam with grad_scale (device scalar, 1 / world: the mean). Bitwise one process learning on the
 * union of the ranks' minibatches when the sums are exact in any order (SharedCriticLearner.dp_learn). Call before
 * the first flock_sc_pipeline_learn. */
typedef int (*FlockAllreduceFn)(void* ctx, float* data, int64_t n, void* learner_stream);
int flock_sc_pipeline_set_dp(FlockScPipeline* p, float* bucket, int64_t critic_floats, int64_t actor_off,
                             int64_t bucket_floats, const float* grad_scale, FlockAllreduceFn allreduce, void* ctx);
/* The actor half of each data-parallel round off the learner chain (after flock_sc_pipeline_set_dp, before the first
 * learn): slot i's actor gradient goes to actor_grads[i] (one actor's floats, 16-B aligned, one buffer per slot), and
 * its all-reduce (`allreduce(ctx, actor_grads[i], actor_floats, actor_stream)`, e.g. over a second process group) and
 * Adam step run on a stream of the pipeline's own, behind an event for the round's gradient launches; only the critic
 * all-reduce and the critic Adam stay on learner_stream, whose next critic phase needs them, and of the critic all-reduce
 * only the fc1 / LayerNorm-1 part [0, fc2.weight offset) follows the gradient launch: the rest, complete after the bwd
 * launch, is all-reduced (first `allreduce` call of the round, on a third stream of the pipeline's own) while the
 * gradient launch runs. Every later reader of
 * that agent's actor on learner_stream (its next learn: 256 learns later at config 3) waits for the actor step's
 * event unless the host already sees it complete; flush joins the actor stream into learner_stream. Bitwise the
 * unsplit rounds (agent_simple_shared_critic.py:137-150; the reference steps the actor right after the critic). */
int flock_sc_pipeline_set_dp_actor(FlockScPipeline* p, float* const* actor_grads, int n_agents,
                                   FlockAllreduceFn allreduce, void* ctx);
/* The pipeline's own comm stream (split data-parallel rounds: the early critic all-reduce), NULL before
 * flock_sc_pipeline_set_dp_actor: lets a caller bind one collective communicator to each stream that calls it. */
void* flock_sc_pipeline_comm_stream(const FlockScPipeline* p);

#ifdef __cplusplus
}
#endif

#endif /* FLOCK_LEARN_H */
