// flock_torch_sc.h — shared-critic argument lists of the torch layer (csrc/flock_torch_learn.cpp), shared with the
// training-loop classes (csrc/flock_torch_loop.cpp).
//   learner = [critic, critic_grad, critic_exp_avg, critic_exp_avg_sq, critic_step [1] i64, actors, actors_grad,
//              actors_exp_avg, actors_exp_avg_sq, actors_target, actor_steps [n_agents] i64, losses [2], counters [2] i32]
//   job     = [idx [B] i64, agent [1] i64, state, new_state, action, reward, terminal, workspace, critic_view
//              (empty: none)(, actor_grad_out)]
//   dims    = [B, in_dim, n_actions, fc1, fc2, update_rate, do_adam]; hyper = [alpha, beta, gamma, beta1, beta2, eps, tau]
#pragma once

#include <ATen/ATen.h>

#include "flock_learn.h"

namespace flock_torch {

// TORCH_CHECKs of one job (empty: only the learner state) against the learner state, dims and hyper
void sc_round_checks(at::TensorList L, at::TensorList job, at::IntArrayRef dims, at::ArrayRef<double> hyper,
                     const char* what);
// the FlockScUpdate of one job
FlockScUpdate sc_update(at::TensorList L, at::TensorList job, at::IntArrayRef dims, at::ArrayRef<double> hyper);

}  // namespace flock_torch
