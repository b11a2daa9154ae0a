/*
 * rlks_oracle.c — CPU restatement of the reference environment (TEST INFRASTRUCTURE ONLY).
 *
 * This file is the parity CHECKER for the HIP path.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product path (librlks.so) never links it.
 *
 * What it restates, line by line of /root/reference/rl_scheduler/env/k8s_multi_cloud_env.py:
 *   _get_live_cpu  (:84-88)   random.uniform(0.1, 0.8) = 0.1 + (0.8-0.1) * random()
 *   _get_obs       (:90-103)  f32[ cost[0..C), lat[0..C), cpu[0..C) ] of row current_step
 *   reset          (:106-112) current_step = 0; random.seed(seed) when seed is given
 *   step           (:115-144) validate; reward = 100*(0.6*cost + 0.4*lat) of row t (f64, no FMA);
 *                             t += 1; done = t >= max_steps; obs of row t (IndexError past T-1)
 * plus CPython's MT19937 (Modules/_randommodule.c: init_genrand, init_by_array, genrand_uint32,
 * random_random = genrand_res53) for the bit-exact "compat" noise mode, and Philox4x32-10
 * (Salmon et al., SC'11; Random123) for the counter-based mode.
 *
 * Pinned by tests/test_oracle_golden.py against tests/golden/ (generated from the reference env
 * itself by tools/make_goldens.py).  Build: see oracle/Makefile (gcc -O2 -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rlks_types.h"

#if defined(__FP_FAST_FMA)
#error "oracle must be built with -ffp-contract=off (reward must not be FMA-contracted)"
#endif

/* --------------------------------------------------------------------------- Philox4x32-10 */
void ro_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* n counters ctr[n][4] -> out[n][4] */
void ro_philox_batch(const uint32_t* ctr, const uint32_t key[2], uint32_t* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) ro_philox4x32_10(ctr + 4 * i, key, out + 4 * i);
}

/* 53-bit uniform in [0,1) from two 32-bit words, CPython genrand_res53's construction */
double ro_u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

/* --------------------------------------------------------------------------- MT19937 */
#define MT_N 624
#define MT_M 397
/* state layout: mt[0..623], mt[624] = mti */
static void mt_init_genrand(uint32_t* mt, uint32_t s) {
  mt[0] = s;
  for (int i = 1; i < MT_N; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
  mt[MT_N] = MT_N;
}

void ro_mt_seed(uint32_t* mt, const uint32_t* key, int keylen) {
  mt_init_genrand(mt, 19650218u);
  int i = 1, j = 0;
  int k = MT_N > keylen ? MT_N : keylen;
  for (; k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
    ++i; ++j;
    if (i >= MT_N) { mt[0] = mt[MT_N - 1]; i = 1; }
    if (j >= keylen) j = 0;
  }
  for (k = MT_N - 1; k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
    ++i;
    if (i >= MT_N) { mt[0] = mt[MT_N - 1]; i = 1; }
  }
  mt[0] = 0x80000000u;
  mt[MT_N] = MT_N;
}

uint32_t ro_mt_u32(uint32_t* mt) {
  static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
  uint32_t y;
  if (mt[MT_N] >= MT_N) {
    int kk;
    for (kk = 0; kk < MT_N - MT_M; ++kk) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < MT_N - 1; ++kk) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    y = (mt[MT_N - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
    mt[MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 1u];
    mt[MT_N] = 0;
  }
  y = mt[mt[MT_N]++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

double ro_mt_random(uint32_t* mt) {
  uint32_t a = ro_mt_u32(mt), b = ro_mt_u32(mt);
  return ro_u53(a, b);
}

/* --------------------------------------------------------------------------- batched env */
typedef struct ro_env {
  rlks_env_cfg cfg;
  double* cost; /* [T][C] */
  double* lat;  /* [T][C] */
  int32_t* step;
  int32_t* episode;
  uint32_t* mt; /* [n][625] */
  /* node-level extension; NULL / 0 when nodes_per_cluster == 0 */
  int32_t* cap_cpu;   /* [C] millicores per node */
  int32_t* cap_mem;   /* [C] MiB per node */
  int32_t* init_max;  /* [C] max initial pods per node = floor(init_occupancy * max_pods) */
  int32_t* free_cpu;  /* [n][C][N] */
  int32_t* free_mem;  /* [n][C][N] */
  int32_t* used_cpu;  /* [n][C] */
  double* lam;        /* arrival rates: [1] (Poisson) or [n_trace] (bursty) */
  double* enl;        /* exp(-lam), computed once on the host */
  int n_trace;
  int maxp;           /* most pods a node can hold */
  uint32_t* skip;     /* [n_skip] geometric survival (1 - depart_prob)^j in units of 2^-32 */
  int n_skip;
  int64_t counters[6]; /* node checks, pods placed, pods rejected, pods departed, node write-backs,
                          node reads */
} ro_env;

ro_env* ro_env_create(const rlks_env_cfg* cfg, const double* cost, const double* lat) {
  if (!cfg || cfg->n_envs <= 0 || cfg->n_rows <= 0 || cfg->n_clouds <= 0) return NULL;
  ro_env* e = (ro_env*)calloc(1, sizeof(ro_env));
  e->cfg = *cfg;
  size_t tc = (size_t)cfg->n_rows * cfg->n_clouds, n = (size_t)cfg->n_envs;
  e->cost = (double*)malloc(tc * sizeof(double));
  e->lat = (double*)malloc(tc * sizeof(double));
  memcpy(e->cost, cost, tc * sizeof(double));
  memcpy(e->lat, lat, tc * sizeof(double));
  e->step = (int32_t*)calloc(n, sizeof(int32_t));
  e->episode = (int32_t*)calloc(n, sizeof(int32_t));
  e->mt = (uint32_t*)calloc(n * (MT_N + 1), sizeof(uint32_t));
  for (size_t i = 0; i < n; ++i) {
    uint64_t s = cfg->seed + (uint64_t)(cfg->env_offset + (int64_t)i); /* random.seed(seed + global id) */
    uint32_t key[2] = {(uint32_t)s, (uint32_t)(s >> 32)};
    ro_mt_seed(e->mt + i * (MT_N + 1), key, key[1] ? 2 : 1);
  }
  return e;
}

void ro_env_destroy(ro_env* e) {
  if (!e) return;
  free(e->cost); free(e->lat); free(e->step); free(e->episode); free(e->mt);
  free(e->cap_cpu); free(e->cap_mem); free(e->init_max); free(e->free_cpu); free(e->free_mem);
  free(e->used_cpu); free(e->lam); free(e->enl); free(e->skip);
  free(e);
}

/* ---------------------------------------------------------------- node-level extension
 * Spec (builder-defined, the reference has no node state).  Per env, C clusters
 * x N nodes with integer free millicores / MiB; homogeneous pods (req_cpu, req_mem).
 *  reset: node g = c*N + n gets pods0 = (x * (init_max[c] + 1)) >> 32 with x = word (g & 3) of
 *         Philox(ctr = {gid, episode, g >> 2, OCCUPANCY << 16}).
 *  step(a) at row t:
 *   1. departures (every running pod leaves independently with probability p =
 *      depart_prob), realised per cluster as geometric skips over the cluster's P pods (numbered in
 *      node order at the start of the step), so that a step reads only clusters where a pod leaves:
 *      for c = 0..C-1 with P = used_cpu[c] / req_cpu > 0 (and p > 0): pos = 0, k = 0; while pos < P:
 *      u = word (k & 3) of Philox({gid, episode, t | (k >> 2) << 16, DEPART << 16 | c}), k++;
 *      R = P - pos; if u < S(R) stop (none of the remaining R pods leaves); else s = #{j in [1,
 *      min(R, L)) : S(j) > u} pods survive and pod pos + s leaves; pos += s + 1.  S = ro_skip32(p)
 *      (length L; S(j) = 0 for j >= L) is the survival table round((1 - p)^j 2^32), capped at
 *      2^32 - 1, so P(s >= j) = (1 - p)^j: the departing set has the per-pod Bernoulli(p) law.
 *      The pod's node is found by scanning the cluster's nodes in order (pods per node as at the
 *      start of the step); its free cpu / mem grow by one request;
 *   2. arrivals: k ~ Poisson(lam) by inverse transform on u53 of Philox({gid, episode, t,
 *      ARRIVAL << 16}) words (0, 1): p = exp(-lam); F = p; while (u > F && k < 64)
 *      { k++; p = p * lam / k; F += p; }  (f64, no FMA; lam = rate, or trace[t mod n_trace]);
 *   3. first-fit: each pod goes to the lowest-index node of cluster a with free cpu >= req_cpu
 *      and free mem >= req_mem (the scan resumes where the previous pod landed); none -> rejected;
 *   4. reward = scale * (w_cost * cost[t][a] + w_lat * lat[t][a]) - penalty * rejected;
 *   5. t += 1; obs = [cost[t][.], lat[t][.], (float)used_cpu[c] / (float)(N * cap_cpu[c])].
 *  counters: [0] first-fit node checks, [1] placed, [2] rejected, [3] departed, [4] node write-backs
 *  (one per node that lost pods, one per node that received pods), [5] 8-node chunks read (those
 *  holding departing pods; first fit: the chunks up to the last one tried, except chunks whose 8
 *  nodes are all full, which the device skips by its per-chunk pod totals). */

/* Survival table of the departure skips: S[j] = round((1 - p)^j * 2^32) capped at 2^32 - 1, for
 * j = 0 .. n - 1 where n = min(pmax, first j with S[j] == 0) + 1 (entries past the table are 0).
 * Plain f64 multiplies in this order.  Returns n (out may be NULL to size the table). */
int ro_skip32(int pmax, double p, uint32_t* out) {
  const double q = 1.0 - p;
  double acc = 1.0;
  int n = 0;
  for (int j = 0; j <= pmax; ++j) {
    double x = acc * 4294967296.0;
    x = x + 0.5;
    const uint32_t v = x >= 4294967295.0 ? 0xffffffffu : (uint32_t)x;
    if (v == 0u) break;
    if (out) out[j] = v;
    n = j + 1;
    acc = acc * q;
  }
  return n;
}

static void nodes_reset_lane(ro_env* e, int lane) {
  const rlks_env_cfg* cfg = &e->cfg;
  const int C = cfg->n_clouds, N = cfg->nodes_per_cluster;
  int32_t* fc = e->free_cpu + (size_t)lane * C * N;
  int32_t* fm = e->free_mem + (size_t)lane * C * N;
  int32_t* used = e->used_cpu + (size_t)lane * C;
  uint32_t key[2] = {(uint32_t)cfg->seed, (uint32_t)(cfg->seed >> 32)};
  for (int c = 0; c < C; ++c) used[c] = 0;
  for (int g = 0; g < C * N; ++g) {
    uint32_t x[4];
    uint32_t ctr[4] = {(uint32_t)(cfg->env_offset + lane), (uint32_t)e->episode[lane], (uint32_t)(g >> 2),
                       (uint32_t)RLKS_PURPOSE_OCCUPANCY << 16};
    ro_philox4x32_10(ctr, key, x);
    const int c = g / N;
    const int32_t pods = (int32_t)(((uint64_t)x[g & 3] * (uint64_t)(e->init_max[c] + 1)) >> 32);
    fc[g] = e->cap_cpu[c] - pods * cfg->pod_cpu_m;
    fm[g] = e->cap_mem[c] - pods * cfg->pod_mem_mi;
    used[c] += pods * cfg->pod_cpu_m;
  }
}

/* returns rejected pods */
static int nodes_step_lane(ro_env* e, int lane, int a, int t) {
  const rlks_env_cfg* cfg = &e->cfg;
  const int C = cfg->n_clouds, N = cfg->nodes_per_cluster;
  int32_t* fc = e->free_cpu + (size_t)lane * C * N;
  int32_t* fm = e->free_mem + (size_t)lane * C * N;
  int32_t* used = e->used_cpu + (size_t)lane * C;
  uint32_t key[2] = {(uint32_t)cfg->seed, (uint32_t)(cfg->seed >> 32)};
  const uint32_t gid = (uint32_t)(cfg->env_offset + lane), ep = (uint32_t)e->episode[lane];
  const double pdep = cfg->depart_prob;
  for (int c = 0; c < C && pdep > 0.0; ++c) {
    const int P = used[c] / cfg->pod_cpu_m;
    int32_t* cfc = fc + (size_t)c * N;
    int32_t* cfm = fm + (size_t)c * N;
    int pos = 0, k = 0, n = 0, cum = 0, dn = 0;  /* node scan: n, pods before it, departures from it */
    int seen = -1;                                /* last 8-node chunk holding a departing pod */
    uint32_t x[4] = {0, 0, 0, 0};
    while (pos < P) {
      if ((k & 3) == 0) {
        uint32_t ctr[4] = {gid, ep, (uint32_t)t | ((uint32_t)(k >> 2) << 16),
                           ((uint32_t)RLKS_PURPOSE_DEPART << 16) | (uint32_t)c};
        ro_philox4x32_10(ctr, key, x);
      }
      const uint32_t u = x[k & 3];
      ++k;
      const int R = P - pos;
      const uint32_t sR = R < e->n_skip ? e->skip[R] : 0u;
      if (u < sR) break;
      int s = 0;
      const int lim = R < e->n_skip ? R : e->n_skip;
      while (s + 1 < lim && e->skip[s + 1] > u) ++s;
      const int idx = pos + s;
      pos = idx + 1;
      /* node of pod idx: advance the scan, writing back the node left behind */
      for (;;) {
        const int pn = (e->cap_cpu[c] - cfc[n]) / cfg->pod_cpu_m + dn; /* pods at the start of the step */
        if (idx < cum + pn) break;
        if (dn) { e->counters[4] += 1; dn = 0; }
        cum += pn;
        ++n;
      }
      if ((n >> 3) != seen) { e->counters[5] += 1; seen = n >> 3; }
      cfc[n] += cfg->pod_cpu_m;
      cfm[n] += cfg->pod_mem_mi;
      used[c] -= cfg->pod_cpu_m;
      ++dn;
      e->counters[3] += 1;
    }
    if (dn) e->counters[4] += 1;
  }
  uint32_t x[4];
  uint32_t ctr[4] = {gid, ep, (uint32_t)t, (uint32_t)RLKS_PURPOSE_ARRIVAL << 16};
  ro_philox4x32_10(ctr, key, x);
  const double u = ro_u53(x[0], x[1]);
  const int j = cfg->arrival_mode ? t % e->n_trace : 0;
  const double lam = e->lam[j];
  double p = e->enl[j], F = p;
  int k = 0;
  while (u > F && k < 64) {
    k += 1;
    p = p * lam / (double)k;
    F = F + p;
  }
  int n = 0, rejected = 0, last = -1;
  int32_t* ac = fc + (size_t)a * N;
  int32_t* am = fm + (size_t)a * N;
  int32_t* ac_start = (int32_t*)malloc((size_t)N * sizeof(int32_t)); /* free cpu before the arrivals */
  memcpy(ac_start, ac, (size_t)N * sizeof(int32_t));
  for (int i = 0; i < k; ++i) {
    while (n < N && !(ac[n] >= cfg->pod_cpu_m && am[n] >= cfg->pod_mem_mi)) ++n;
    e->counters[0] += (n < N) ? 1 : 0;
    if (n == N) { rejected = k - i; break; }
    if (n != last) { e->counters[4] += 1; last = n; }
    ac[n] -= cfg->pod_cpu_m;
    am[n] -= cfg->pod_mem_mi;
    used[a] += cfg->pod_cpu_m;
    e->counters[1] += 1;
  }
  e->counters[0] += n;
  e->counters[2] += rejected;
  { /* first-fit chunk reads: the 8-node chunks the scan reaches with pods left to place, except
       those whose nodes are all full (skipped by their pod totals) */
    int mp = e->cap_cpu[a] / cfg->pod_cpu_m;
    if (e->cap_mem[a] / cfg->pod_mem_mi < mp) mp = e->cap_mem[a] / cfg->pod_mem_mi;
    const int last_ch = k == 0 ? -1 : (rejected ? N / 8 - 1 : n >> 3);
    for (int ch = 0; ch <= last_ch; ++ch) {
      int full = 1;
      for (int q = 0; q < 8; ++q) {
        const int node = 8 * ch + q;
        /* fullness when the scan reached the chunk: before it (ch < n >> 3 and not rejected) the
           chunk is full now iff it was then (first fit placed nothing there) */
        if ((e->cap_cpu[a] - ac_start[node]) / cfg->pod_cpu_m < mp) full = 0;
      }
      if (!full) e->counters[5] += 1;
    }
  }
  free(ac_start);
  return rejected;
}

int ro_env_enable_nodes(ro_env* e, const int32_t* cap_cpu, const int32_t* cap_mem, const double* lam,
                        int n_trace) {
  const rlks_env_cfg* cfg = &e->cfg;
  const int C = cfg->n_clouds, N = cfg->nodes_per_cluster;
  const size_t n = (size_t)cfg->n_envs;
  if (N <= 0 || cfg->pod_cpu_m <= 0 || cfg->pod_mem_mi <= 0) return -1;
  e->cap_cpu = (int32_t*)malloc(C * sizeof(int32_t));
  e->cap_mem = (int32_t*)malloc(C * sizeof(int32_t));
  e->init_max = (int32_t*)malloc(C * sizeof(int32_t));
  for (int c = 0; c < C; ++c) {
    e->cap_cpu[c] = cap_cpu[c];
    e->cap_mem[c] = cap_mem[c];
    int mp = cap_cpu[c] / cfg->pod_cpu_m;
    if (cap_mem[c] / cfg->pod_mem_mi < mp) mp = cap_mem[c] / cfg->pod_mem_mi;
    e->init_max[c] = (int32_t)floor(cfg->init_occupancy * (double)mp);
    if (e->init_max[c] > mp) e->init_max[c] = mp;
    if (mp > e->maxp) e->maxp = mp;
  }
  if (e->maxp > 64 || N % 8 != 0 || (long)C * N > 262144 || cfg->n_rows > 65535 || C > 1024) return -1;
  e->n_skip = ro_skip32(N * e->maxp, cfg->depart_prob, NULL);
  e->skip = (uint32_t*)malloc((size_t)(e->n_skip > 0 ? e->n_skip : 1) * sizeof(uint32_t));
  ro_skip32(N * e->maxp, cfg->depart_prob, e->skip);
  e->n_trace = cfg->arrival_mode ? n_trace : 1;
  e->lam = (double*)malloc(e->n_trace * sizeof(double));
  e->enl = (double*)malloc(e->n_trace * sizeof(double));
  for (int i = 0; i < e->n_trace; ++i) {
    e->lam[i] = cfg->arrival_mode ? lam[i] : cfg->arrival_rate;
    e->enl[i] = exp(-e->lam[i]);
  }
  e->free_cpu = (int32_t*)calloc(n * C * N, sizeof(int32_t));
  e->free_mem = (int32_t*)calloc(n * C * N, sizeof(int32_t));
  e->used_cpu = (int32_t*)calloc(n * C, sizeof(int32_t));
  for (size_t i = 0; i < n; ++i) nodes_reset_lane(e, (int)i);
  return 0;
}

void ro_env_node_state(const ro_env* e, int32_t* free_cpu, int32_t* free_mem, int32_t* used_cpu) {
  const size_t n = (size_t)e->cfg.n_envs, CN = (size_t)e->cfg.n_clouds * e->cfg.nodes_per_cluster;
  if (free_cpu) memcpy(free_cpu, e->free_cpu, n * CN * sizeof(int32_t));
  if (free_mem) memcpy(free_mem, e->free_mem, n * CN * sizeof(int32_t));
  if (used_cpu) memcpy(used_cpu, e->used_cpu, n * e->cfg.n_clouds * sizeof(int32_t));
}

void ro_env_counters(const ro_env* e, int64_t* out6) { memcpy(out6, e->counters, sizeof(e->counters)); }

int ro_env_seed_lane(ro_env* e, int lane, const uint32_t* key, int keylen) {
  if (!e || lane < 0 || lane >= e->cfg.n_envs || keylen <= 0) return -1;
  ro_mt_seed(e->mt + (size_t)lane * (MT_N + 1), key, keylen);
  return 0;
}

int32_t ro_env_lane_step(const ro_env* e, int lane) { return e->step[lane]; }
int32_t ro_env_lane_episode(const ro_env* e, int lane) { return e->episode[lane]; }
void ro_env_lane_counters(const ro_env* e, int32_t* step, int32_t* episode) {
  memcpy(step, e->step, (size_t)e->cfg.n_envs * sizeof(int32_t));
  memcpy(episode, e->episode, (size_t)e->cfg.n_envs * sizeof(int32_t));
}

static double noise_draw(ro_env* e, int lane, int t, int c) {
  const rlks_env_cfg* cfg = &e->cfg;
  double u;
  if (cfg->noise_mode == RLKS_NOISE_MT19937) {
    u = ro_mt_random(e->mt + (size_t)lane * (MT_N + 1));
  } else {
    uint32_t ctr[4] = {(uint32_t)(cfg->env_offset + lane), (uint32_t)e->episode[lane], (uint32_t)t,
                       ((uint32_t)RLKS_PURPOSE_OBS << 16) | (uint32_t)(c >> 1)};
    uint32_t key[2] = {(uint32_t)cfg->seed, (uint32_t)(cfg->seed >> 32)};
    uint32_t x[4];
    ro_philox4x32_10(ctr, key, x);
    u = (c & 1) ? ro_u53(x[2], x[3]) : ro_u53(x[0], x[1]);
  }
  double span = cfg->cpu_hi - cfg->cpu_lo; /* 0.8 - 0.1 = 0.7000000000000001 */
  return cfg->cpu_lo + span * u;
}

/* obs of row t for one lane (consumes C noise draws, AWS first: :92-93) */
static void write_obs(ro_env* e, int lane, int t, float* obs) {
  const int C = e->cfg.n_clouds, N = e->cfg.nodes_per_cluster;
  for (int c = 0; c < C; ++c) obs[c] = (float)e->cost[(size_t)t * C + c];
  for (int c = 0; c < C; ++c) obs[C + c] = (float)e->lat[(size_t)t * C + c];
  if (N > 0) {
    for (int c = 0; c < C; ++c)
      obs[2 * C + c] = (float)e->used_cpu[(size_t)lane * C + c] / (float)(N * e->cap_cpu[c]);
  } else {
    for (int c = 0; c < C; ++c) obs[2 * C + c] = (float)noise_draw(e, lane, t, c);
  }
}

int ro_env_reset(ro_env* e, const uint8_t* mask, float* obs) {
  const int D = 3 * e->cfg.n_clouds;
  for (int i = 0; i < e->cfg.n_envs; ++i) {
    if (mask && !mask[i]) continue;
    e->step[i] = 0;
    e->episode[i] += 1;
    if (e->cfg.nodes_per_cluster > 0) nodes_reset_lane(e, i);
    write_obs(e, i, 0, obs + (size_t)i * D);
  }
  return 0;
}

/*
 * status[0] = invalid actions (nothing steps when > 0: the reference asserts before any change)
 * status[1] = lanes that ran past the table (reference IndexError from iloc, :91 via :144)
 */
int ro_env_step(ro_env* e, const int32_t* actions, float* obs, double* reward, uint8_t* term,
                int32_t* step_out, float* final_obs, int32_t* status) {
  const rlks_env_cfg* cfg = &e->cfg;
  const int C = cfg->n_clouds, T = cfg->n_rows, D = 3 * C;
  status[0] = status[1] = 0;
  for (int i = 0; i < cfg->n_envs; ++i)
    if (actions[i] < 0 || actions[i] >= C) status[0]++;
  if (status[0]) return 0;
  for (int i = 0; i < cfg->n_envs; ++i) {
    const int a = actions[i];
    int t = e->step[i];
    term[i] = 0;
    if (t >= T) { status[1]++; reward[i] = 0.0; step_out[i] = t; continue; }
    int rejected = cfg->nodes_per_cluster > 0 ? nodes_step_lane(e, i, a, t) : 0;
    double cost = e->cost[(size_t)t * C + a];
    double lat = e->lat[(size_t)t * C + a];
    double t1 = cfg->w_cost * cost;
    double t2 = cfg->w_lat * lat;
    reward[i] = cfg->scale * (t1 + t2);
    if (cfg->reject_penalty != 0.0) reward[i] = reward[i] - cfg->reject_penalty * (double)rejected;
    t += 1;
    e->step[i] = t;
    step_out[i] = t;
    int done = t >= cfg->max_steps;
    term[i] = (uint8_t)done;
    if (t >= T) { status[1]++; continue; }
    float* o = obs + (size_t)i * D;
    write_obs(e, i, t, o);
    if (done && cfg->autoreset) {
      if (final_obs) memcpy(final_obs + (size_t)i * D, o, D * sizeof(float));
      e->step[i] = 0;
      e->episode[i] += 1;
      if (cfg->nodes_per_cluster > 0) nodes_reset_lane(e, i);
      write_obs(e, i, 0, o);
    }
  }
  return 0;
}
