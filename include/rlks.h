/*
 * rlks.h — C ABI of librlks.so, the MI355X (gfx950) rollout-and-training engine for the
 * rl_scheduler multi-cloud pod scheduler.
 *
 * Drop-in boundary.  The reference's hot path sits behind the gymnasium Env API
 * (K8sMultiCloudEnv, /root/reference/rl_scheduler/env/k8s_multi_cloud_env.py:36-157) and behind
 * RLlib's PPO Algorithm surface (train(), compute_single_action(), save()/from_checkpoint(),
 * /root/reference/rl_scheduler/agent/train_ppo.py:9-31, eval_ppo.py:17-27,
 * final_evaluation.py:32-48).  The Python host package (rl-k8s-scheduler_amd/rlks) keeps that
 * surface and binds the entry points below with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Every function returns 0 (RLKS_OK) or a negative RLKS_ERR_* code; rlks_last_error() gives
 *    the message (thread-local).
 *  - Pointers named *_dev are device (HBM) pointers owned by the caller (torch tensors);
 *    *_host pointers are host memory.  `stream` is a hipStream_t (NULL = legacy default stream).
 *  - All device work is enqueued asynchronously on `stream`; no function synchronises the
 *    device except rlks_env_create/destroy, so every call can be captured in a hipGraph.
 *  - Handles are not re-entrant: one handle per GPU per host thread.
 */
#ifndef RLKS_H
#define RLKS_H

#include <stdint.h>

#include "rlks_types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RLKS_OK 0
#define RLKS_ERR_ARG (-1)
#define RLKS_ERR_HIP (-2)
#define RLKS_ERR_UNSUPPORTED (-3)
#define RLKS_ERR_STATE (-4)

const char* rlks_last_error(void);
const char* rlks_version(void);

/* Debug build only (make -C csrc debug -> librlks_debug.so): device-side bounds checks that count
 * instead of faulting.  out[3] = {violations since the last call, first site (rlks_internal.h
 * DcheckSite), its value}; synchronises the device and clears the counters.  RLKS_ERR_UNSUPPORTED
 * in the product library. */
int rlks_debug_checks(unsigned long long* out);

/* ============================================================== environment (K1 + K2) ==== */
typedef struct rlks_env rlks_env;

/* K8sMultiCloudEnv.__init__ (:46-66): tables are [n_rows][n_clouds] float64 host arrays with the
 * exact bits pandas parsed from data/processed/normalized_rl_data.csv (:58).  Allocates the SoA
 * lane state (step, episode, optional MT19937 state) in HBM.  Synchronises. */
int rlks_env_create(const rlks_env_cfg* cfg, const double* cost_host, const double* lat_host,
                    rlks_env** out);
/* Same, with the node-level extension when cfg->nodes_per_cluster > 0: node_cpu_m
 * and node_mem_mi are per-cluster node capacities [n_clouds]; arrival_trace [n_trace] gives the
 * per-step Poisson rate for arrival_mode 1 (bursty), indexed by step mod n_trace. */
int rlks_env_create_ext(const rlks_env_cfg* cfg, const double* cost_host, const double* lat_host,
                        const int32_t* node_cpu_m_host, const int32_t* node_mem_mi_host,
                        const double* arrival_trace_host, int n_trace, rlks_env** out);
int rlks_env_destroy(rlks_env* env);
int rlks_env_config(const rlks_env* env, rlks_env_cfg* out);

/* random.seed(seed) (:109-110) for the lanes in mask (NULL = all), MT19937 mode only:
 * keys_dev[lane * key_stride + j] are the 32-bit words of abs(seed), little-endian (CPython
 * random_seed); keylen_dev[lane] is the word count (>= 1). */
int rlks_env_seed(rlks_env* env, const uint8_t* mask_dev, const uint32_t* keys_dev,
                  const int32_t* keylen_dev, int key_stride, void* stream);

/* Advance each masked lane's MT19937 stream by n_draws_dev[lane] random() calls (int64 per lane;
 * MT19937 mode only).  Batched evaluation uses it to give lane e the stream position of episode e
 * of the reference's sequential loop (final_evaluation.py:42-49, one process-global generator). */
int rlks_env_mt_discard(rlks_env* env, const uint8_t* mask_dev, const int64_t* n_draws_dev, void* stream);
/* Lane's MT19937 state as CPython's random.getstate()[1] lays it out: 624 words then the position
 * (0..624), copied to (to_env = 0) or from (to_env = 1) words_dev[625] (MT19937 mode only).  The
 * drop-in env's "global" noise stream keeps the lane in step with the process-global `random`
 * module this way: the reference draws its cpu noise from it (k8s_multi_cloud_env.py:87) and
 * reseeds it in reset (:109-111). */
int rlks_env_mt_words(rlks_env* env, int lane, uint32_t* words_dev, int to_env, void* stream);

/* reset() (:106-112) for the lanes in mask (NULL = all): current_step = 0, obs of row 0. */
int rlks_env_reset(rlks_env* env, const uint8_t* mask_dev, float* obs_dev, void* stream);

/* step(action) (:115-144) for all lanes.  status_dev[0] = invalid actions (when > 0 NO lane
 * steps: the reference asserts before any change, :116); status_dev[1] = lanes that ran past the
 * last table row (the reference's IndexError, :91).  reward64 is bit-exact f64 (no FMA);
 * reward32 its f32 rounding; one of the two reward pointers, truncated, step_out and final_obs
 * may be NULL.  Node-level envs (nodes_per_cluster > 0)
 * run the node sweep (departures, arrivals, first-fit) in the same call.
 * status_dev == NULL declares the actions trusted (produced by rlks sampling): no validation
 * launch and no status report. */
int rlks_env_step(rlks_env* env, const int32_t* actions_dev, float* obs_dev, double* reward64_dev,
                  float* reward32_dev, uint8_t* terminated_dev, uint8_t* truncated_dev,
                  int32_t* step_out_dev, float* final_obs_dev, int32_t* status_dev, void* stream);

/* Fused action sampling + step for the rollout (RLlib sampler + TorchCategorical): action =
 * Categorical(logits) via Philox (explore != 0) or argmax (explore == 0, compute_single_action
 * explore=False); logp of the chosen action; env step; auto-reset; episode-return tracking.
 * Table envs only (RLKS_ERR_UNSUPPORTED for node-level envs). */
int rlks_env_sample_step(rlks_env* env, const float* logits_dev, int explore, int32_t* actions_dev,
                         float* logp_dev, float* obs_next_dev, float* reward_dev, uint8_t* done_dev,
                         void* stream);

/* TorchCategorical sample (explore != 0) or argmax of rows i < n of logits_dev[n][A]: the draw of
 * row i is Philox4x32-10 of the counter {ids[3i], ids[3i + 1], ids[3i + 2], RLKS_PURPOSE_ACTION << 16}
 * under key = seed, turned into an action exactly as rlks_env_sample_step does (ids may be NULL
 * when explore = 0); logp_dev (may be NULL) gets log pi(action).  compute_single_action(obs) with
 * exploration (eval_ppo.py:27) keys its draw by (config seed, call counter). */
int rlks_sample_categorical(const float* logits_dev, int n, int A, const uint32_t* ids_dev, unsigned long long seed,
                            int explore, int32_t* actions_dev, float* logp_dev, void* stream);

/* Sum of completed-episode returns and their count over all lanes (double[2]); clear != 0
 * zeroes the accumulators (PPO result "episode_reward_mean", train_ppo.py:29-30). */
int rlks_env_episode_stats(rlks_env* env, double* out_dev, int clear, void* stream);

/* Completed-episode log since the last clear: returns_dev[RLKS_EPLOG_CAP] (float64) and
 * keys_dev[RLKS_EPLOG_CAP] (int64: episode << 32 | global lane) of the first RLKS_EPLOG_CAP
 * episodes, count_dev[0] (uint32) = all episodes completed (may exceed the capacity).  Sorting by
 * key gives completion order.  Feeds RLlib's 100-episode smoothing of episode_reward_mean
 * (metrics_num_episodes_for_smoothing; train_ppo.py:29-30 prints it).  Any pointer may be NULL. */
int rlks_env_episode_log(rlks_env* env, double* returns_dev, long long* keys_dev, unsigned* count_dev,
                         int clear, void* stream);

/* Snapshot of every per-lane state a resumed run needs (step / episode counters, episode returns,
 * MT19937 words, node free cpu / mem and per-cluster used cpu): rlks_env_state_bytes gives the
 * size; save / load copy it to / from a device buffer of that size, asynchronously on `stream`.
 * Checkpoint / resume (agent.save() each iteration, train_ppo.py:31;
 * PPO.from_checkpoint, eval_ppo.py:17).  Philox draws are keyed by (lane, episode, step), so the
 * counters restore the random streams too. */
int rlks_env_state_bytes(const rlks_env* env, int64_t* bytes);
int rlks_env_save_state(const rlks_env* env, void* dst_dev, void* stream);
int rlks_env_load_state(rlks_env* env, const void* src_dev, void* stream);

/* node-level extension: free millicores / MiB per node as [n_envs][n_clouds][nodes] and the
 * per-cluster used millicores [n_envs][n_clouds] (any pointer may be NULL) */
int rlks_env_node_state(rlks_env* env, int32_t* free_cpu_dev, int32_t* free_mem_dev, int32_t* used_cpu_dev,
                        void* stream);
/* node counters {node checks by first fit, pods placed, pods rejected, pods departed, node
 * write-backs, node reads} (u64[6]) copied to out_dev when non-NULL; enable = 1 / 0 turns counting on (zeroed) / off, -1
 * leaves it unchanged.  The flag is read when a step is launched (a captured graph keeps it). */
int rlks_env_counters(rlks_env* env, int enable, unsigned long long* out_dev, void* stream);

/* copy lane counters (current_step, episode index) into caller buffers (either may be NULL) */
int rlks_env_lane_state(rlks_env* env, int32_t* steps_dev, int32_t* episodes_dev, void* stream);

/* ============================================================== RNG test surface ========= */
/* Philox4x32-10 of n counters ctr_dev[n][4] under key_dev[2] -> out_dev[n][4] */
int rlks_philox4x32_10(const uint32_t* ctr_dev, const uint32_t* key_dev, uint32_t* out_dev, int n,
                       void* stream);
/* n draws of CPython random.random() after random.seed(key words) -> out_dev[n] (one lane) */
int rlks_mt_random(const uint32_t* key_dev, int keylen, double* out_dev, int n, void* stream);

/* ============================================================== advantages (K3) ========== */
/* RLlib compute_advantages (use_gae=True) over a time-major [T][N] rollout:
 *   delta_t = r_t + gamma * V_{t+1} * (1 - done_t) - V_t,  A_t = delta_t + gamma*lam*(1-done_t)*A_{t+1}
 *   vtarg_t = A_t + V_t;  values_dev is [T+1][N] (row T = bootstrap V(s_T)).
 * partials_dev (may be NULL) receives per-block [sum A, sum A^2] for standardisation. */
int rlks_gae(const float* rewards_dev, const float* values_dev, const uint8_t* dones_dev, float gamma,
             float lam, int T, int N, float* adv_dev, float* vtarg_dev, double* partials_dev,
             void* stream);
int rlks_gae_partials_count(int N);
/* sums_dev[3] = {sum A, sum A^2, count} from the partials (deterministic order) */
int rlks_adv_stats(const double* partials_dev, int n_partials, double count, double* sums_dev,
                   void* stream);
/* dyn_dev[ADV_MEAN], dyn_dev[ADV_INVSTD] from (possibly all-reduced) sums (numpy std, ddof=0) */
int rlks_adv_finalize(const double* sums_dev, float* dyn_dev, void* stream);

/* ============================================================== policy / value MLP (K4) == */
/* Flat parameter buffer layout (fp32, torch [out][in] weights, each tensor 64-float aligned).
 * Tensor indices (offsets12[i]):
 *   0 pi.w1 [H][D]  1 pi.b1 [H]  2 pi.w2 [H][H]  3 pi.b2 [H]  4 pi.w3 [A][H]  5 pi.b3 [A]
 *   6 vf.w1 [H][D]  7 vf.b1 [H]  8 vf.w2 [H][H]  9 vf.b2 [H] 10 vf.w3 [1][H] 11 vf.b3 [1]
 * stored in the order 0 1 6 7 2 3 4 5 8 9 10 11 (both nets' first layers first: the two gradient
 * buckets of rlks_ppo_grad_step_part are [0, offsets12[2]) and [offsets12[2], padded)).
 * (RLlib FCNet with vf_share_layers=False: _hidden_layers/_logits/_value_branch_separate/
 *  _value_branch.) */
#define RLKS_N_TENSORS 12
int rlks_mlp_layout(const rlks_mlp_desc* desc, int64_t* offsets12, int64_t* padded_count,
                    int64_t* real_count);

/* logits_dev[n][A], values_dev[n] = FCNet forward of obs_dev[n][D] (either output may be NULL) */
int rlks_policy_forward(const rlks_mlp_desc* desc, const float* params_dev, const float* obs_dev,
                        int n, float* logits_dev, float* values_dev, void* stream);

/* Rollout buffers, time-major, device pointers */
typedef struct rlks_rollout_bufs {
  float* obs;       /* [T+1][N][D] */
  float* logits;    /* [T][N][A] */
  float* values;    /* [T+1][N] */
  int32_t* actions; /* [T][N] */
  float* logp;      /* [T][N] */
  float* rewards;   /* [T][N] */
  uint8_t* dones;   /* [T][N] */
  float* adv;       /* [T][N] */
  float* vtarg;     /* [T][N] */
  int32_t T;
  int32_t N;
  int32_t global_lanes; /* lanes of the whole data-parallel job (0: N).  The split-fp16 rollout picks
                           its forward kernel from this count, not from N, so that a lane's rollout
                           does not depend on how the job's lanes are split over ranks. */
} rlks_rollout_bufs;

/* T steps of (policy forward -> sample -> env step) into bufs, then the bootstrap values
 * V(obs[T]).  obs[0] must hold the current observations. */
int rlks_rollout(rlks_env* env, const rlks_mlp_desc* desc, const float* params_dev,
                 const rlks_rollout_bufs* bufs, int explore, void* stream);
/* Policy / value forward with a workspace (rlks_ppo_workspace_bytes for >= n rows): required for
 * the generic-width path (RLKS_PRECISION_WIDE or shapes outside the fused kernels). */
int rlks_policy_forward_ws(const rlks_mlp_desc* desc, const float* params_dev, const float* obs_dev, int n,
                           float* logits_dev, float* values_dev, void* workspace, int64_t ws_bytes, void* stream);
/* Generic split-fp16 GEMM of the wide-MLP path (config c5); see rlks_gemm_desc. */
int rlks_gemm_sf16(const rlks_gemm_desc* desc, void* stream);
/* atomicMax of max |x| over x[rows][cols] (row stride ld) into *slot (caller zeroes the slot). */
int rlks_absmax(const float* x, int rows, int cols, int ld, uint32_t* slot, void* stream);
/* Same rollout; with desc->precision == RLKS_PRECISION_SF16 it runs the split-fp16 step kernel
 * (both nets' forward + sample + env step per launch, values written per step, V(obs[T]) last)
 * with the split weights in `workspace` (an rlks_ppo_workspace_bytes-sized buffer: the SGD step's
 * workspace can be shared).  Other precisions fall through to rlks_rollout. */
int rlks_rollout_ws(rlks_env* env, const rlks_mlp_desc* desc, const float* params_dev,
                    const rlks_rollout_bufs* bufs, int explore, void* workspace, int64_t ws_bytes,
                    void* stream);

/* Minibatch rows per packed record: [obs D | logits_old A | adv | vtarg | logp_old | action] */
int rlks_minibatch_stride(const rlks_mlp_desc* desc);
/* Gather minibatch rows [row0, row0+rows) of epoch `epoch`'s permutation of the T*N samples
 * (Philox-keyed Feistel bijection, no sort) into mb_dev; advantages standardised with dyn. */
int rlks_ppo_gather(const rlks_mlp_desc* desc, const rlks_rollout_bufs* bufs, uint64_t perm_seed,
                    int epoch, int64_t row0, int rows, const float* dyn_dev, float* mb_dev,
                    void* stream);
/* Same over `groups` equal blocks of lanes (global block ids group0 .. group0 + groups - 1): block
 * k has its own permutation of its T * (N / groups) samples and supplies rows / groups rows of every
 * minibatch (rows [k rows/groups, (k+1) rows/groups) of mb_dev, row0 / groups onwards in its
 * order).  A run on W ranks with one block each then draws exactly the minibatches of a
 * single-rank run over all lanes with W blocks: training is independent of the world size up to
 * fp32 summation order.  groups (<= 64) must divide N, rows and row0.  groups = 1, group0 = 0 is
 * rlks_ppo_gather. */
int rlks_ppo_gather_grouped(const rlks_mlp_desc* desc, const rlks_rollout_bufs* bufs, uint64_t perm_seed,
                            int epoch, int groups, int group0, int64_t row0, int rows, const float* dyn_dev,
                            float* mb_dev, void* stream);
/* Floats per sample record of rlks_ppo_pack: the minibatch record padded to a 64-byte multiple
 * (16 / 32 / 48 for obs 6 / 12 / 24); 0 for shapes the packed path does not cover. */
int rlks_packed_stride(const rlks_mlp_desc* desc);
/* The rollout's T*N samples as records [T*N][rlks_packed_stride] in rollout order (after GAE):
 * one aligned record per sample, so that each minibatch row is one random line read. */
int rlks_ppo_pack(const rlks_mlp_desc* desc, const rlks_rollout_bufs* bufs, float* packed_dev, void* stream);
/* rlks_ppo_gather_grouped from packed records: the same rows, permutation and record bytes. */
int rlks_ppo_gather_packed(const rlks_mlp_desc* desc, const float* packed_dev, int T, int N, uint64_t perm_seed,
                           int epoch, int groups, int group0, int64_t row0, int rows, float* mb_dev, void* stream);

/* Gradient of the RLlib PPO loss (mean over `rows`*world rows via dyn[INV_COUNT]) w.r.t. the
 * flat parameters -> grad_dev (padded_count floats).  stats_dev (double[RLKS_STAT_SIZE]) gets
 * the sums for reporting and the KL update.  workspace from rlks_ppo_workspace_bytes. */
int rlks_ppo_workspace_bytes(const rlks_mlp_desc* desc, int rows, int64_t* bytes);
/* Diagnostics (tools/f1b_isolate.py): the split-fp16 step's dZ2 hand-off inside `workspace` for `rows`
 * minibatch rows: out[net] = dZ2 planes ([rows / 16 tiles][8][hi, lo][64][8] fp16, sgd_sf16.hip F1a),
 * out[2 + net] = the tiles' int32 split exponents. */
int rlks_debug_sf_handoff(const rlks_mlp_desc* desc, int rows, void* workspace_dev, void** out);
/* Diagnostics (tools/wide_b2_isolate.py): the generic-width step's per-net forward and loss buffers
 * inside `workspace` after rlks_ppo_grad: out[3 net] = H2 [rows][hidden], out[3 net + 1] = head
 * outputs [rows][A or 1], out[3 net + 2] = dL/d outputs [rows][A or 1] (float32). */
int rlks_debug_wide_bufs(const rlks_mlp_desc* desc, int rows, void* workspace_dev, void** out);
int rlks_ppo_grad(const rlks_mlp_desc* desc, const rlks_ppo_coeffs* coeffs, const float* params_dev,
                  const float* dyn_dev, const float* mb_dev, int rows, float* grad_dev,
                  double* stats_dev, void* workspace_dev, int64_t workspace_bytes, void* stream);

/* Same, launching only the phases in `phases` (profiling / benchmarking: each phase reads what the
 * previous phases left in the workspace). */
#define RLKS_PHASE_FWD 1    /* F1: forward + head + loss + dZ2 */
#define RLKS_PHASE_DW2 2    /* F2: dW2 = dZ2^T H1 (split over rows) */
#define RLKS_PHASE_DH1 4    /* F3: dH1 = dZ2 W2 -> dZ1 -> dW1, db1 partials */
#define RLKS_PHASE_REDUCE 8 /* fixed-order reduction of all partials (+ stats) */
#define RLKS_PHASE_ALL 15
#define RLKS_PHASE_FWD_PI 16 /* F1 of the policy net only (profiling) */
#define RLKS_PHASE_FWD_VF 32 /* F1 of the value net only (profiling) */
#define RLKS_PHASE_PREP 64   /* split-fp16: weight split/permute (implied by RLKS_PHASE_FWD) */
#define RLKS_PHASE_F1A 128   /* split-fp16, split F1: k_sf_fwd only, both nets (profiling) */
#define RLKS_PHASE_F1B 256   /* split-fp16, split F1: k_sf_bwd only, both nets (profiling) */
int rlks_ppo_grad_phases(const rlks_mlp_desc* desc, const rlks_ppo_coeffs* coeffs, const float* params_dev,
                         const float* dyn_dev, const float* mb_dev, int rows, float* grad_dev, double* stats_dev,
                         void* workspace_dev, int64_t workspace_bytes, int phases, void* stream);

/* In-pipeline kernel timing of the split-fp16 gradient (bench.py roofline): `reps` full rlks_ppo_grad
 * passes on `stream` (after one untimed pass), each kernel launched with a start / stop event pair
 * (hipExtLaunchKernelGGL: the kernel's own duration, as rocprofv3 measures it); ms_out[6] = average ms
 * of the weight split (k_sf_split), F1a (k_sf_fwd; or the fused k_sf_f1, see rlks_sf_f1_fused), F1b
 * (k_sf_bwd; 0 when fused), F2 (k_sf_dw2r) and the reduce (k_reduce), each less the event bracket's own
 * cost, which ms_out[5] reports (the same bracket around an empty kernel).  Synchronises the stream. */
int rlks_ppo_grad_profile(const rlks_mlp_desc* desc, const rlks_ppo_coeffs* coeffs, const float* params_dev,
                          const float* dyn_dev, const float* mb_dev, int rows, float* grad_dev, double* stats_dev,
                          void* workspace_dev, int64_t workspace_bytes, int reps, double* ms_out, void* stream);

/* 1 if a whole split-fp16 gradient of this descriptor runs F1 as one kernel (k_sf_f1: the default up to
 * 4 actions; RLKS_F1_FUSED=1 / RLKS_F1_SPLIT=1 in the environment force either form), else 0 (bench.py
 * names the kernels it times and profiles by it).  Not a reference interface: build introspection. */
int rlks_sf_f1_fused(const rlks_mlp_desc* desc);

/* torch.optim.Adam step (lerp form of exp_avg, bias-corrected), in place on n floats */
int rlks_adam_step(float* params_dev, const float* grad_dev, float* m_dev, float* v_dev, int64_t n,
                   float lr, float beta1, float beta2, float eps, int step, void* stream);
/* One SGD step on one rank: the PPO gradient of the minibatch (as rlks_ppo_grad; `grad` still
 * receives it) with Adam (as rlks_adam_step, step `step`) applied inside the gradient reduction,
 * which also leaves the new weights' max |w| for the next step's operand split (prev_fused = 1 on
 * the step after a fused one: the weight-max pass is skipped, with a device-side check that falls
 * back to scanning the weights).  Replaces rlks_ppo_grad + rlks_adam_step when no gradient
 * all-reduce sits between them; other precisions run exactly those two calls. */
int rlks_ppo_sgd_step(const rlks_mlp_desc* desc, const rlks_ppo_coeffs* coeffs, float* params_dev,
                      const float* dyn_dev, const float* mb_dev, int rows, float* grad_dev, double* stats_dev,
                      float* adam_m_dev, float* adam_v_dev, int64_t n_params, float lr, float beta1, float beta2,
                      float eps, int step, int prev_fused, void* workspace, int64_t ws_bytes, void* stream);

/* rlks_ppo_sgd_step followed by the next step's rlks_ppo_gather_packed (the arguments below) into
 * next->mb_dev, which may be this step's own mb_dev: the gather runs inside the step's last launch
 * (its gradient reduction), after every read of the minibatch.  Same rows and bytes as the two
 * calls; next == NULL is rlks_ppo_sgd_step.  (Reference: RLlib's minibatch loop,
 * sgd_minibatch_size at rl_scheduler/agent/train_ppo.py:16, draws minibatch k+1 after SGD step k.) */
typedef struct rlks_gather_next {
  const float* packed_dev; /* rlks_ppo_pack records [T N] */
  float* mb_dev;
  uint64_t perm_seed;
  int64_t row0;
  int T, N, epoch, groups, group0, rows;
} rlks_gather_next;
int rlks_ppo_sgd_step_next(const rlks_mlp_desc* desc, const rlks_ppo_coeffs* coeffs, float* params_dev,
                           const float* dyn_dev, const float* mb_dev, int rows, float* grad_dev, double* stats_dev,
                           float* adam_m_dev, float* adam_v_dev, int64_t n_params, float lr, float beta1, float beta2,
                           float eps, int step, int prev_fused, const rlks_gather_next* next, void* workspace,
                           int64_t ws_bytes, void* stream);

/* The same SGD step across ranks (reference: RLlib's multi-GPU learner, one gradient all-reduce per
 * minibatch): rlks_ppo_grad_step writes the rank's gradient (as rlks_ppo_grad; its operand split
 * reads the maxima the previous rlks_ppo_adam_apply left when prev_fused = 1); the caller all-reduces
 * grad_dev; rlks_ppo_adam_apply then applies Adam step `step` in place (as rlks_adam_step,
 * bit-identical) and leaves the new weights' maxima for the next step.  `rows` / the workspace are
 * those of the gradient call; n_params = the padded layout size.  Other precisions run
 * rlks_ppo_grad / rlks_adam_step. */
int rlks_ppo_grad_step(const rlks_mlp_desc* desc, const rlks_ppo_coeffs* coeffs, const float* params_dev,
                       const float* dyn_dev, const float* mb_dev, int rows, float* grad_dev, double* stats_dev,
                       int step, int prev_fused, void* workspace, int64_t ws_bytes, void* stream);
/* rlks_ppo_grad_step + the next step's gather, as rlks_ppo_sgd_step_next (the gather blocks ride
 * in the gradient-reduce launch, before the caller's all-reduce). */
int rlks_ppo_grad_step_next(const rlks_mlp_desc* desc, const rlks_ppo_coeffs* coeffs, const float* params_dev,
                            const float* dyn_dev, const float* mb_dev, int rows, float* grad_dev, double* stats_dev,
                            int step, int prev_fused, const rlks_gather_next* next, void* workspace,
                            int64_t ws_bytes, void* stream);
/* rlks_ppo_grad_step_next in two parts, so that the caller's all-reduce of part 1's gradient buckets
 * runs under part 2's kernels: part 1 = the weight split, the forward / loss kernel (F1a), dW2 / db2
 * (F2) and the reduce of W2, b2, W3, b3 (both nets) and the stats; part 2 = the dH1 / dW1 kernel
 * (F1b) and the reduce of W1, b1 (+ the next gather, `next` is read by part 2 only).  The gradient
 * equals rlks_ppo_grad_step's bit for bit.  Buckets (offsets of rlks_mlp_layout, storage order
 * above): part 1 = [off[2], padded), part 2 = [off[0], off[2]), one contiguous range each.  Other
 * precisions: the whole gradient in part 1, part 2 only gathers. */
int rlks_ppo_grad_step_part(const rlks_mlp_desc* desc, const rlks_ppo_coeffs* coeffs, const float* params_dev,
                            const float* dyn_dev, const float* mb_dev, int rows, float* grad_dev, double* stats_dev,
                            int step, int prev_fused, int part, const rlks_gather_next* next, void* workspace,
                            int64_t ws_bytes, void* stream);
int rlks_ppo_adam_apply(const rlks_mlp_desc* desc, float* params_dev, const float* grad_dev, float* adam_m_dev,
                        float* adam_v_dev, int64_t n_params, float lr, float beta1, float beta2, float eps, int step,
                        void* workspace, int64_t ws_bytes, int rows, void* stream);

/* RLlib update_kl: kl = stats_sum[0] / stats_sum[1]; x1.5 if kl > 2*target, x0.5 if < target/2 */
int rlks_kl_update(float* dyn_dev, const double* kl_sum_count_dev, float kl_target, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RLKS_H */
