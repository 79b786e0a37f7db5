/*
 * flock_learn.h — C ABI of the learner-side HIP kernels in libflock_amd.so (gfx950).
 *
 * Device pointers, sizes, scalars; `stream` is a hipStream_t passed as an opaque pointer. Return 0 or a negative
 * code (flock_learn_last_error() holds the message). They replace, for ALL agents of a learner at once:
 *   flock_adam_step    torch.optim.Adam.step() per agent network (learners/maddpg_official_rnn/agent.py:32-33,
 *                      maddpg_shared_critic/ddpg_network.py:273,347, vdn/train_flock.py:265) fused with the
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

/* gather: dst[r][:] = src[idx[r]][:]; scatter: dst[idx[r]][:] = src[r][:]; rows of `width` floats. */
int flock_gather_rows(void* stream, int64_t rows, int64_t width, const float* src, const int64_t* idx, float* dst);
int flock_scatter_rows(void* stream, int64_t rows, int64_t width, const float* src, const int64_t* idx, float* dst);

#ifdef __cplusplus
}
#endif

#endif /* FLOCK_LEARN_H */
