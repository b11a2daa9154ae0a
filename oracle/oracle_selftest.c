/*
 * oracle_selftest.c — drives rlks_oracle.c under AddressSanitizer + UndefinedBehaviorSanitizer
 * (`make -C oracle sanitize`; SURVEY.md §5 "host ASan/UBSan on the CPU restatement").  TEST
 * INFRASTRUCTURE ONLY: run by tests/test_oracle_sanitize.py.
 *
 * usage: oracle_selftest <table.bin>   (float64 [100][2] cost then [100][2] latency)
 * Exercises every oracle entry point: Philox, MT19937 seeding / draws, the batched env in both
 * noise modes with auto-reset and the terminal overrun, and the node-level extension (Poisson and
 * trace arrivals, departures, first-fit).  Prints the round-robin episode return of lane 0 in
 * MT19937 mode (seed 42) and a checksum line; exits non-zero on any inconsistency.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rlks_types.h"

typedef struct ro_env ro_env;
void ro_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
void ro_mt_seed(uint32_t* mt, const uint32_t* key, int keylen);
double ro_mt_random(uint32_t* mt);
ro_env* ro_env_create(const rlks_env_cfg* cfg, const double* cost, const double* lat);
void ro_env_destroy(ro_env* e);
int ro_env_enable_nodes(ro_env* e, const int32_t* cap_cpu, const int32_t* cap_mem, const double* lam, int n_trace);
int ro_env_reset(ro_env* e, const uint8_t* mask, float* obs);
int ro_env_step(ro_env* e, const int32_t* actions, float* obs, double* reward, uint8_t* term, int32_t* step_out,
                float* final_obs, int32_t* status);
void ro_env_node_state(const ro_env* e, int32_t* free_cpu, int32_t* free_mem, int32_t* used_cpu);
void ro_env_counters(const ro_env* e, int64_t* out6);
void ro_env_lane_counters(const ro_env* e, int32_t* step, int32_t* episode);

static rlks_env_cfg cfg_of(int n, int C, int noise, uint64_t seed, int autoreset) {
  rlks_env_cfg c;
  memset(&c, 0, sizeof c);
  c.n_envs = n; c.n_rows = 100; c.n_clouds = C; c.max_steps = 99; c.noise_mode = noise; c.autoreset = autoreset;
  c.seed = seed; c.cpu_lo = 0.1; c.cpu_hi = 0.8; c.w_cost = 0.6; c.w_lat = 0.4; c.scale = 100.0;
  return c;
}

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: %s table.bin\n", argv[0]); return 2; }
  double tab[400];
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(tab, sizeof(double), 400, f) != 400) { fprintf(stderr, "bad table\n"); return 2; }
  fclose(f);
  const double* cost = tab;
  const double* lat = tab + 200;

  /* Philox + MT19937 */
  uint32_t ctr[4] = {0, 0, 0, 0}, key[2] = {0, 0}, out[4];
  ro_philox4x32_10(ctr, key, out);
  uint32_t mt[625];
  uint32_t k42 = 42;
  ro_mt_seed(mt, &k42, 1);
  double s = 0.0;
  for (int i = 0; i < 2000; ++i) s += ro_mt_random(mt);

  /* reference env in MT19937 mode: lane 0 seeded like random.seed(42), round-robin policy
   * (train_and_compare.py:65), one 99-step episode, then one step past the table */
  rlks_env_cfg c = cfg_of(4, 2, RLKS_NOISE_MT19937, 42, 0);
  ro_env* e = ro_env_create(&c, cost, lat);
  float obs[4 * 6], fin[4 * 6];
  double rew[4];
  uint8_t term[4];
  int32_t st[4], status[2], acts[4];
  ro_env_reset(e, NULL, obs);
  double ret = 0.0;
  for (int t = 0; t < 99; ++t) {
    for (int i = 0; i < 4; ++i) acts[i] = t % 2;
    ro_env_step(e, acts, obs, rew, term, st, fin, status);
    if (status[0] || status[1]) { fprintf(stderr, "unexpected status at %d\n", t); return 1; }
    ret += rew[0];
  }
  if (!term[0]) { fprintf(stderr, "episode did not terminate\n"); return 1; }
  ro_env_step(e, acts, obs, rew, term, st, fin, status);  /* iloc[99] + obs of row 100: overrun */
  if (status[1] != 4) { fprintf(stderr, "expected 4 overruns, got %d\n", status[1]); return 1; }
  acts[2] = 7;
  ro_env_step(e, acts, obs, rew, term, st, fin, status);
  if (status[0] != 1) { fprintf(stderr, "invalid action not counted\n"); return 1; }
  ro_env_destroy(e);

  /* Philox mode with auto-reset over 250 steps */
  c = cfg_of(4, 2, RLKS_NOISE_PHILOX, 7, 1);
  e = ro_env_create(&c, cost, lat);
  ro_env_reset(e, NULL, obs);
  double rs = 0.0;
  for (int t = 0; t < 250; ++t) {
    for (int i = 0; i < 4; ++i) acts[i] = (t + i) & 1;
    ro_env_step(e, acts, obs, rew, term, st, fin, status);
    for (int i = 0; i < 4; ++i) rs += rew[i];
  }
  int32_t lst[4], lep[4];
  ro_env_lane_counters(e, lst, lep);
  if (lep[0] != 3 || lst[0] != 250 - 2 * 99) { fprintf(stderr, "lane counters %d %d\n", lep[0], lst[0]); return 1; }
  ro_env_destroy(e);

  /* node-level extension: 8 clusters x 16 nodes, Poisson and trace arrivals */
  double lam_tr[5] = {0.0, 0.5, 1.5, 3.0, 2.0};
  int32_t cap_cpu[8], cap_mem[8];
  for (int k = 0; k < 8; ++k) { cap_cpu[k] = 2000; cap_mem[k] = (k & 1) ? 4096 : 1024; }
  double cost8[800], lat8[800];
  for (int i = 0; i < 800; ++i) { cost8[i] = cost[(i / 8) * 2 + (i & 1)]; lat8[i] = lat[(i / 8) * 2 + (i & 1)]; }
  int64_t cnt_total = 0;
  for (int mode = 0; mode < 2; ++mode) {
    c = cfg_of(6, 8, RLKS_NOISE_PHILOX, 3, 1);
    c.nodes_per_cluster = 16; c.pod_cpu_m = 100; c.pod_mem_mi = 64; c.arrival_mode = mode; c.arrival_rate = 4.0;
    c.depart_prob = 0.05; c.init_occupancy = 0.5; c.reject_penalty = 0.1;
    e = ro_env_create(&c, cost8, lat8);
    if (ro_env_enable_nodes(e, cap_cpu, cap_mem, lam_tr, 5)) { fprintf(stderr, "enable_nodes failed\n"); return 1; }
    float o8[6 * 24], f8[6 * 24];
    double r8[6];
    uint8_t t8[6];
    int32_t s8[6], a8[6];
    ro_env_reset(e, NULL, o8);
    for (int t = 0; t < 220; ++t) {
      for (int i = 0; i < 6; ++i) a8[i] = (t * 3 + i) % 8;
      ro_env_step(e, a8, o8, r8, t8, s8, f8, status);
    }
    int32_t fc[6 * 8 * 16], fm[6 * 8 * 16], used[6 * 8];
    ro_env_node_state(e, fc, fm, used);
    for (int i = 0; i < 6; ++i)
      for (int k = 0; k < 8; ++k) {
        int32_t u = 0;
        for (int n = 0; n < 16; ++n) {
          const int32_t x = fc[(i * 8 + k) * 16 + n], y = fm[(i * 8 + k) * 16 + n];
          if (x < 0 || y < 0 || x > cap_cpu[k] || y > cap_mem[k]) { fprintf(stderr, "node out of range\n"); return 1; }
          if ((cap_cpu[k] - x) / 100 != (cap_mem[k] - y) / 64) { fprintf(stderr, "cpu/mem pods disagree\n"); return 1; }
          u += cap_cpu[k] - x;
        }
        if (u != used[i * 8 + k]) { fprintf(stderr, "used aggregate mismatch\n"); return 1; }
      }
    int64_t cnt[6];
    ro_env_counters(e, cnt);
    cnt_total += cnt[1] + cnt[3];
    ro_env_destroy(e);
  }
  printf("round_robin_return %.17g\n", ret);
  printf("checksum %u %.17g %.17g %lld\n", out[0], s, rs, (long long)cnt_total);
  return 0;
}
