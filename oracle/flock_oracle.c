/*
 * flock_oracle.c — CPU ORACLE (test infrastructure, NOT product code).
 *
 * A plain-C restatement of the reference environments' step() hot path, used only by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg, always as the checker / the timed CPU
 * port — never as the product path. The product path is the HIP library in marl_range_flocking_amd/csrc.
 *
 * Parity is PINNED: tests/test_oracle_golden.py checks every function here against golden vectors produced by
 * running the reference itself (tests/golden/gen_golden_env.py imports /root/reference on torch CPU).
 *
 * Conventions (shared with the HIP kernels, and the reason they are bit-exact against this file):
 *   * float32 everywhere, every op rounded separately (built with -ffp-contract=off: no FMA fusion), in the
 *     reference's op order;
 *   * kNN order: ascending (d2, j), d2 = fl(fl(dx*dx) + fl(dy*dy)); this is a valid tie resolution of the
 *     reference's topk(-sqrt(d2), k+1) (sqrt is monotone), whose own tie order is implementation-defined;
 *     returned distances are the correctly-rounded sqrt of the winners' d2;
 *   * per-env float sums (centre of mass, mean heading) use a fixed power-of-two tree order
 *     (buf[i] += buf[i + s], s = P/2 .. 1), the order the GPU's LDS reduction uses.
 * Transcendentals (cosf/sinf) come from libm; the GPU uses ocml. They may differ by an ulp, which is why the
 * step tests compare float state with rtol 1e-5 and check the kNN stage bit-exactly on identical positions.
 *
 * Layouts (row-major, contiguous): pos [E][N][2], heading/prev [E][N], action [E][N][2] (f32) or [E][N] (i64),
 * vel [E][N][2], dnn [E][N][k], idx [E][N][k] (i64), reward [E][N], done [E][N] (u8), any_done [E] (u8),
 * obs memory [E][N][4][k].
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

#define MEM 4 /* observation memory depth, gym_flock_uw.py:59, gym_flock.py:42 */

static float clampf_t(float x, float lo, float hi) {
    /* torch.clamp(x, lo, hi): NaN propagates */
    if (x < lo) return lo;
    if (x > hi) return hi;
    return x;
}

static float nan_to_num(float x) { /* torch.nan_to_num defaults */
    if (isnan(x)) return 0.0f;
    if (isinf(x)) return x > 0 ? FLT_MAX : -FLT_MAX;
    return x;
}

/* check_boundary(), gym_flock_v2.py:271-304 (identical in all four envs). Non-rigid = teleport, not modulo. */
static void boundary(float* p, float box, int rigid) {
    for (int c = 0; c < 2; ++c) {
        float v = p[c];
        if (rigid) {
            v = (v < box) ? v : box;  /* :274-278 */
            v = (v > 0.0f) ? v : 0.0f; /* :279-281 */
        } else {
            v = (v < box) ? v : 0.001f; /* :292-294 */
            v = (v > 0.0f) ? v : box;   /* :295-297 */
        }
        p[c] = v;
    }
}

static float tree_sum(const float* v, int n, float* buf) {
    int P = 1;
    while (P < n) P <<= 1;
    for (int i = 0; i < P; ++i) buf[i] = (i < n) ? v[i] : 0.0f;
    for (int s = P >> 1; s >= 1; s >>= 1)
        for (int i = 0; i < s; ++i) buf[i] = buf[i] + buf[i + s];
    return buf[0];
}

/* Pair distance squared. Periodic: gym_flock_v2.py:137-144 (|xi-xj|, B-d if d > B/2, mul, mul, add).
 * Euclidean: the torch.norm of gym_flock_v2.py:166 restated as fl(fl(dx*dx)+fl(dy*dy)). */
static float pair_d2(float xi, float yi, float xj, float yj, float box, int periodic) {
    float dx = xi - xj, dy = yi - yj;
    if (periodic) {
        float half = box * 0.5f;
        dx = fabsf(dx);
        dy = fabsf(dy);
        dx = (dx > half) ? (box - dx) : dx;
        dy = (dy > half) ? (box - dy) : dy;
    }
    float sx = dx * dx;
    float sy = dy * dy;
    return sx + sy;
}

/*
 * kNN of every agent: topk(-D, k+1) then drop rank 0 (self), gym_flock_v2.py:147-151 / :171-175.
 * clamp != 0 → distances clamped to [0, sensor_range] (v2/uw/uw_discrete); 0 → unclamped (gym_flock.py:105).
 * Returns -1 if k+1 > N (the reference's topk raises "selected index k out of range").
 */
/* normalize_distance=True of the reference constructors (test switch, set by oracle.py around a call): the
 * Euclidean kNN runs on positions / max_i torch.norm(p_i) of each env (gym_flock_v2.py:157-163, gym_flock_uw.py:127-133,
 * gym_flock_uw_discrete.py:175-181, gym_flock.py:94-98). The periodic kNN never normalises. */
static int g_normalize = 0;
void oracle_set_normalize(int on) { g_normalize = on != 0; }

int oracle_knn(int E, int N, int k, float box, float sensor_range, int periodic, int clamp,
               const float* pos, float* dnn, int64_t* idx) {
    if (k + 1 > N || k < 1) return -1;
    int L = k + 1;
    float* bd = (float*)malloc(sizeof(float) * L);
    int* bj = (int*)malloc(sizeof(int) * L);
    float* qn = (float*)malloc(sizeof(float) * 2 * (size_t)N);
    for (int e = 0; e < E; ++e) {
        const float* P = pos + (size_t)e * N * 2;
        if (g_normalize && !periodic) {
            float m = 0.0f;
            for (int i = 0; i < N; ++i) {
                float sx = P[2 * i] * P[2 * i], sy = P[2 * i + 1] * P[2 * i + 1];
                float n = sqrtf(sx + sy); /* torch.norm(positions, dim=1) */
                m = (n > m) ? n : m;       /* torch.max(magnitudes) */
            }
            for (int i = 0; i < 2 * N; ++i) qn[i] = P[i] / m; /* positions / max */
            P = qn;
        }
        for (int i = 0; i < N; ++i) {
            int cnt = 0;
            for (int j = 0; j < N; ++j) {
                float d2 = pair_d2(P[2 * i], P[2 * i + 1], P[2 * j], P[2 * j + 1], box, periodic);
                /* strict '<' with ascending j keeps the lower index first among equal d2 */
                if (cnt < L || d2 < bd[L - 1]) {
                    int s = (cnt < L) ? cnt++ : L - 1;
                    while (s > 0 && d2 < bd[s - 1]) {
                        bd[s] = bd[s - 1];
                        bj[s] = bj[s - 1];
                        --s;
                    }
                    bd[s] = d2;
                    bj[s] = j;
                }
            }
            size_t o = ((size_t)e * N + i) * k;
            for (int s = 1; s < L; ++s) {
                float d = sqrtf(bd[s]);
                if (clamp) d = clampf_t(d, 0.0f, sensor_range);
                dnn[o + s - 1] = d;
                idx[o + s - 1] = bj[s];
            }
        }
    }
    free(bd);
    free(bj);
    free(qn);
    return 0;
}

/* collisions + dones: _computeCollisions gym_flock_v2.py:212-215, _computeDone :306-315 */
static void collide(int E, int N, int k, float cd, const float* dnn, uint8_t* done, uint8_t* any_done) {
    for (int e = 0; e < E; ++e) {
        uint8_t any = 0;
        for (int i = 0; i < N; ++i) {
            uint8_t c = 0;
            const float* d = dnn + ((size_t)e * N + i) * k;
            for (int s = 0; s < k; ++s) c |= (d[s] < cd);
            done[(size_t)e * N + i] = c;
            any |= c;
        }
        any_done[e] = any;
    }
}

/* obs memory roll + insert: torch.roll(mem, 1, dims=1); mem[:,0,:] = dnn (gym_flock_uw.py:120-123) */
static void mem_roll(int E, int N, int k, const float* mem_in, const float* dnn, float* mem_out) {
    for (size_t a = 0; a < (size_t)E * N; ++a) {
        const float* mi = mem_in + a * MEM * k;
        float* mo = mem_out + a * MEM * k;
        /* descending s: also correct when mem_in == mem_out */
        for (int s = MEM - 1; s >= 1; --s)
            for (int c = 0; c < k; ++c) mo[s * k + c] = mi[(s - 1) * k + c];
        for (int c = 0; c < k; ++c) mo[c] = dnn[a * k + c];
    }
}

/*
 * gym_flock_v2.MultiAgentEnv.step (gym_flock_v2.py:71-83). periodic=1 is the reference env; periodic=0 with
 * v_min=0.5 is the fork learners/maddpg_official_rnn/gym_flock_v2.py:71-82 (Euclidean, :310).
 */
int oracle_step_v2(int E, int N, int k, float box, float sensor_range, float cd, float dt, float v_min,
                   float v_max, int periodic, int rigid, float* pos, float* heading, const float* action,
                   float* vel, float* dnn, int64_t* idx, float* reward, uint8_t* done, uint8_t* any_done) {
    if (k + 1 > N || k < 1) return -1;
    const float half_pi = (float)(M_PI / 2.0);
    for (size_t a = 0; a < (size_t)E * N; ++a) {
        float lin = action[2 * a], ang = action[2 * a + 1]; /* :324-325 */
        ang = clampf_t(ang, -half_pi, half_pi);             /* :327 */
        float t = ang * dt;
        heading[a] = heading[a] + t;                        /* :329 */
        lin = clampf_t(lin, v_min, v_max);                  /* :331 */
        float h = heading[a];
        float vx = lin * cosf(h);                           /* :335 */
        float vy = lin * sinf(h);                           /* :336 */
        vx = nan_to_num(vx);                                /* :346 */
        vy = nan_to_num(vy);
        vx = vx * dt;                                       /* :349 */
        vy = vy * dt;
        vel[2 * a] = vx;
        vel[2 * a + 1] = vy;
        pos[2 * a] = pos[2 * a] + vx;                       /* :350 */
        pos[2 * a + 1] = pos[2 * a + 1] + vy;
        boundary(pos + 2 * a, box, rigid);                  /* :74 → :271-304 */
    }
    oracle_knn(E, N, k, box, sensor_range, periodic, 1, pos, dnn, idx); /* :76 → :135-151 */
    collide(E, N, k, cd, dnn, done, any_done);
    for (size_t a = 0; a < (size_t)E * N; ++a) reward[a] = done[a] ? -5.0f : 0.01f; /* :217-220, :268 */
    return 0;
}

/* gym_flock_uw.MultiAgentEnv.step (gym_flock_uw.py:69-81); heading=False kinematics :291-302. */
int oracle_step_uw(int E, int N, int k, float box, float sensor_range, float cd, float dt, int rigid,
                   float* pos, const float* heading, float* prev_heading, const float* action,
                   const float* mem_in, float* mem_out, float* vel, float* dnn, int64_t* idx, float* reward,
                   uint8_t* done, uint8_t* any_done) {
    if (k + 1 > N || k < 1) return -1;
    for (size_t a = 0; a < (size_t)E * N; ++a) {
        float vx = action[2 * a], vy = action[2 * a + 1];     /* :292 */
        float n = sqrtf(vx * vx + vy * vy);                    /* :294 torch.norm(dim=1) */
        vx = vx / n;
        vy = vy / n;
        vx = nan_to_num(vx);                                   /* :298 */
        vy = nan_to_num(vy);
        vx = vx * dt;                                          /* :301 */
        vy = vy * dt;
        vel[2 * a] = vx;
        vel[2 * a + 1] = vy;
        pos[2 * a] = pos[2 * a] + vx;                          /* :302 */
        pos[2 * a + 1] = pos[2 * a + 1] + vy;
        boundary(pos + 2 * a, box, rigid);
    }
    oracle_knn(E, N, k, box, sensor_range, 0, 1, pos, dnn, idx); /* :74 → :125-144 */
    collide(E, N, k, cd, dnn, done, any_done);
    mem_roll(E, N, k, mem_in, dnn, mem_out);                      /* :77 → :120-123 */
    int P = 1;
    while (P < N) P <<= 1;
    float* buf = (float*)malloc(sizeof(float) * P);
    float* xs = (float*)malloc(sizeof(float) * N);
    float* ys = (float*)malloc(sizeof(float) * N);
    const float com_r = cd * 4.0f;
    for (int e = 0; e < E; ++e) {
        for (int i = 0; i < N; ++i) {
            xs[i] = pos[((size_t)e * N + i) * 2];
            ys[i] = pos[((size_t)e * N + i) * 2 + 1];
        }
        float cx = tree_sum(xs, N, buf) / (float)N; /* torch.mean(positions, dim=0) :193 */
        float cy = tree_sum(ys, N, buf) / (float)N;
        for (int i = 0; i < N; ++i) {
            size_t a = (size_t)e * N + i;
            float r = done[a] ? -5.0f : 0.01f;                    /* :186-189 */
            float dx = xs[i] - cx, dy = ys[i] - cy;
            float dist = sqrtf(dx * dx + dy * dy);                /* :194-196 */
            float com = (dist < com_r) ? 0.01f : 0.0f;            /* :197 */
            float diff = fabsf(prev_heading[a] - heading[a]);     /* :202 */
            float angp = (diff > 0.27f) ? -0.01f : 0.001f;        /* :204 */
            prev_heading[a] = heading[a];                         /* :203 */
            reward[a] = (r + com) + angp;                          /* :220 */
        }
    }
    free(buf);
    free(xs);
    free(ys);
    return 0;
}

/*
 * gym_flock_uw_discrete.MultiAgentEnv.step (gym_flock_uw_discrete.py:110-122), _updateState :324-366.
 * table [n_actions][2] = action_dictionary means (:59-75); noise [E][N][2] = the N(0, 0.1) draws that
 * torch.normal adds to the means (:333-334). action ids outside [0, n_actions) return -2 (KeyError in the ref).
 */
int oracle_step_uwd(int E, int N, int k, float box, float sensor_range, float cd, float dt, float v_max,
                    int rigid, float* pos, float* heading, float* prev_heading, const int64_t* action,
                    const float* noise, const float* table, int n_actions, float* vel, float* dnn, int64_t* idx,
                    float* reward, uint8_t* done, uint8_t* any_done) {
    if (k + 1 > N || k < 1) return -1;
    for (size_t a = 0; a < (size_t)E * N; ++a)
        if (action[a] < 0 || action[a] >= n_actions) return -2;
    for (size_t a = 0; a < (size_t)E * N; ++a) {
        int64_t id = action[a];
        float lin = table[2 * id] + noise[2 * a];             /* :329, :333 */
        float ang = table[2 * id + 1] + noise[2 * a + 1];     /* :330, :334 */
        ang = clampf_t(ang, -0.025f, 0.025f);                 /* :343 */
        float t = ang * dt;
        heading[a] = heading[a] + t;                          /* :345 */
        lin = clampf_t(lin, 5e-6f, v_max);                    /* :347 */
        float h = heading[a];
        float vx = lin * cosf(h);                             /* :351 */
        float vy = lin * sinf(h);                             /* :352 */
        float n = sqrtf(vx * vx + vy * vy);                   /* :358 */
        vx = vx / n;
        vy = vy / n;
        vx = nan_to_num(vx);                                  /* :362 */
        vy = nan_to_num(vy);
        vx = vx * dt;                                         /* :365 */
        vy = vy * dt;
        vel[2 * a] = vx;
        vel[2 * a + 1] = vy;
        pos[2 * a] = pos[2 * a] + vx;                         /* :366 */
        pos[2 * a + 1] = pos[2 * a + 1] + vy;
        boundary(pos + 2 * a, box, rigid);
    }
    oracle_knn(E, N, k, box, sensor_range, 0, 1, pos, dnn, idx); /* :115 → :173-192 */
    collide(E, N, k, cd, dnn, done, any_done);
    int P = 1;
    while (P < N) P <<= 1;
    float* buf = (float*)malloc(sizeof(float) * P);
    for (int e = 0; e < E; ++e) {
        float mean_h = tree_sum(heading + (size_t)e * N, N, buf) / (float)N; /* :256 */
        for (int i = 0; i < N; ++i) {
            size_t a = (size_t)e * N + i;
            float coll = done[a] ? -9.0f : 0.0f;                   /* :237 (int64 -9/0) */
            float err = fabsf(mean_h - heading[a]);                /* :257 */
            float align = (err > 0.2f) ? 0.0f : 0.1f;              /* :258 */
            reward[a] = coll + align;                              /* :275 */
            prev_heading[a] = heading[a];                          /* :270 → :251 side effect */
        }
    }
    free(buf);
    return 0;
}

/* gym_flock.MultiAgentEnv.step (gym_flock.py:48-60); _updateState :194-200 (no nan_to_num, no clamp). */
int oracle_step_flock(int E, int N, int k, float box, float cd, float dt, int rigid, float* pos, float* vel,
                      const float* action, const float* mem_in, float* mem_out, float* dnn, int64_t* idx,
                      float* reward, uint8_t* done, uint8_t* any_done) {
    if (k + 1 > N || k < 1) return -1;
    for (size_t a = 0; a < (size_t)E * N; ++a) {
        float tx = action[2 * a] * dt, ty = action[2 * a + 1] * dt;
        float vx = vel[2 * a] + tx, vy = vel[2 * a + 1] + ty;   /* :196 */
        float n = sqrtf(vx * vx + vy * vy);                      /* :198 */
        vx = vx / n;
        vy = vy / n;
        vel[2 * a] = vx;
        vel[2 * a + 1] = vy;
        float sx = vx * dt, sy = vy * dt;
        pos[2 * a] = pos[2 * a] + sx;                            /* :200 */
        pos[2 * a + 1] = pos[2 * a + 1] + sy;
        boundary(pos + 2 * a, box, rigid);
    }
    oracle_knn(E, N, k, box, 0.0f, 0, 0, pos, dnn, idx); /* :53 → :92-105 (no clamp) */
    collide(E, N, k, cd, dnn, done, any_done);
    mem_roll(E, N, k, mem_in, dnn, mem_out);
    for (size_t a = 0; a < (size_t)E * N; ++a) reward[a] = done[a] ? -5.0f : 0.01f; /* :142-145 */
    return 0;
}

int oracle_version(void) { return 1; }
