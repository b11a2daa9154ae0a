/*
 * rlks_types.h — plain-C types shared by the HIP library (librlks.so) and the CPU oracle.
 *
 * The environment model is the reference's K8sMultiCloudEnv
 * (/root/reference/rl_scheduler/env/k8s_multi_cloud_env.py:36-157), generalised to C clouds
 * and batched over n_envs independent lanes.  With n_clouds = 2 and nodes_per_cluster = 0
 * it is the reference env exactly.  nodes_per_cluster > 0 enables
 * the node-level extension specified in DESIGN.md §4 (no reference exists).
 */
#ifndef RLKS_TYPES_H
#define RLKS_TYPES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* cpu-noise / randomness source for the observation's utilisation entries */
enum {
  RLKS_NOISE_PHILOX = 0,   /* Philox4x32-10, key = seed, counter = (env, episode, t, purpose) */
  RLKS_NOISE_MT19937 = 1   /* per-lane CPython MT19937 (random.seed / random.random), bit-exact */
};

/* completed-episode log capacity (rlks_env_episode_log): RLlib smooths episode_reward_mean over at
 * least the last 100 episodes (metrics_num_episodes_for_smoothing), so 100+ individual returns per
 * iteration are all a host ever needs */
enum { RLKS_EPLOG_CAP = 128 };

/* Philox counter purposes (ctr[3] high half) */
enum {
  RLKS_PURPOSE_OBS = 1,
  RLKS_PURPOSE_ACTION = 2,
  RLKS_PURPOSE_ARRIVAL = 3,
  RLKS_PURPOSE_DEPART = 4,
  RLKS_PURPOSE_OCCUPANCY = 5
};

typedef struct rlks_env_cfg {
  int32_t n_envs;        /* lanes */
  int32_t n_rows;        /* T: table rows (reference: 100, normalized_rl_data.csv) */
  int32_t n_clouds;      /* C: clusters / actions (reference: 2, :51) */
  int32_t max_steps;     /* episode length; reference: len(table) - 1 = 99 (:66) */
  int32_t noise_mode;    /* RLKS_NOISE_* */
  int32_t autoreset;     /* 1: terminated lanes reset inside step (vector-env semantics) */
  int32_t env_offset;    /* global id of lane 0 (multi-GPU shard base; Philox counter word 0) */
  int32_t skip_returns;  /* 1: no episode-return bookkeeping in the step (ep_ret / ret_sum / ep_cnt /
                            episode log untouched): the plain gymnasium step contract */
  uint64_t seed;         /* Philox key; also the default MT seed when none is given */
  double cpu_lo;         /* random.uniform(0.1, 0.8) (:87) */
  double cpu_hi;
  double w_cost;         /* reward = scale * (w_cost * cost + w_lat * latency)  (:122) */
  double w_lat;
  double scale;
  /* ---- node-level extension; nodes_per_cluster == 0 disables it ---- */
  int32_t nodes_per_cluster; /* N nodes per cluster */
  int32_t pod_cpu_m;         /* pod request, millicores (simple-service.yaml:27: 100m) */
  int32_t pod_mem_mi;        /* pod request, MiB (simple-service.yaml:28: 64Mi) */
  int32_t arrival_mode;      /* 0: Poisson(arrival_rate); 1: bursty trace (per-step rates) */
  double arrival_rate;       /* mean pod arrivals per step */
  double depart_prob;        /* per-step probability that a running pod leaves (every pod) */
  double init_occupancy;     /* initial pods per node ~ U(0, init_occupancy * max_pods) */
  double reject_penalty;     /* subtracted from reward per rejected pod (0: reference reward) */
} rlks_env_cfg;

/* Multi-layer-perceptron policy/value description (RLlib FCNet, vf_share_layers=False) */
typedef struct rlks_mlp_desc {
  int32_t obs_dim;   /* D  (reference: 6) */
  int32_t hidden;    /* H  (reference: fcnet_hiddens [256, 256]) */
  int32_t n_actions; /* A  (reference: 2) */
  int32_t precision; /* RLKS_PRECISION_*: how the SGD step's matrix products are computed */
} rlks_mlp_desc;

/* SGD-step matrix arithmetic.  Both meet the 1e-5 relative gradient bar against the fp64 oracle:
 * FP32 runs v_mfma_f32_32x32x2_f32 (bitwise an fmaf chain); SF16 splits every operand into two
 * scaled fp16 halves and accumulates three v_mfma_f32_32x32x16_f16 products in fp32 (error
 * <= ~2^-21 per product, measured below the fp32 chain's) at 16x the fp32 matrix rate. */
enum {
  RLKS_PRECISION_FP32 = 0,
  RLKS_PRECISION_SF16 = 1,
  RLKS_PRECISION_WIDE = 2, /* generic split-fp16 GEMM path (wide_mlp.hip): any width, node envs;
                              chosen automatically when the fused 256-unit kernels do not fit */
  RLKS_PRECISION_F16 = 3   /* throughput mode: the split-fp16 SGD kernels with one product (fp16
                              operands hi x hi, fp32 accumulation) instead of three -- below the
                              reference's fp32, a secondary figure only; rollouts as RLKS_PRECISION_SF16 */
};

/* One split-fp16 GEMM (fp32 in / fp32 out, fp32-accurate): C = epi(op(A) op(B)), op = transpose
 * when trans_*; operand scales come from max|x| slots (uint bits of a non-negative float). */
enum {
  RLKS_GEMM_STORE = 0,     /* C = acc */
  RLKS_GEMM_TANH_BIAS = 1, /* C = tanh(acc + bias[n]) */
  RLKS_GEMM_BIAS = 2,      /* C = acc + bias[n] */
  RLKS_GEMM_DTANH = 3      /* C = acc * (1 - aux[m][n]^2) */
};
typedef struct rlks_gemm_desc {
  const float* a;
  const float* b;
  float* c;
  const float* bias;
  const float* aux;
  int32_t m, n, k, lda, ldb, ldc, ldaux;
  int32_t trans_a, trans_b, epilogue, accumulate, reserved;
  const uint32_t* a_max;
  const uint32_t* b_max;
  uint32_t* c_max;         /* optional (NULL): atomicMax of |C| */
} rlks_gemm_desc;

/* PPO loss coefficients that stay fixed for a run (RLlib PPOConfig names and defaults) */
typedef struct rlks_ppo_coeffs {
  float clip_param;      /* 0.3 */
  float vf_clip_param;   /* 10.0 */
  float vf_loss_coeff;   /* 1.0 */
  float entropy_coeff;   /* 0.0 */
} rlks_ppo_coeffs;

/* Device-resident per-iteration scalars (float[RLKS_DYN_SIZE]); kernels read them so that no
 * host round trip is needed between rollout, advantage standardisation and the SGD steps. */
enum {
  RLKS_DYN_ADV_MEAN = 0,    /* mean of the train batch's advantages */
  RLKS_DYN_ADV_INVSTD = 1,  /* 1 / max(1e-4, std)  (RLlib standardize_fields) */
  RLKS_DYN_KL_COEFF = 2,    /* adaptive KL coefficient (initial 0.2) */
  RLKS_DYN_INV_COUNT = 3,   /* 1 / global minibatch rows: the loss is a mean */
  RLKS_DYN_SIZE = 8
};

/* Per-minibatch loss statistics written by rlks_ppo_grad (double[RLKS_STAT_SIZE], sums) */
enum {
  RLKS_STAT_POLICY_LOSS = 0, /* sum of -surrogate */
  RLKS_STAT_VF_LOSS = 1,     /* sum of clipped squared error */
  RLKS_STAT_KL = 2,          /* sum of KL(old || new) */
  RLKS_STAT_ENTROPY = 3,     /* sum of entropy */
  RLKS_STAT_ROWS = 4,        /* rows */
  RLKS_STAT_SIZE = 8
};

#ifdef __cplusplus
}
#endif
#endif /* RLKS_TYPES_H */
