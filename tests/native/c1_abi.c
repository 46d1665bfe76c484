/*
 * c1_abi.c -- a C host of libsiddhi_hip.so written against include/siddhi_hip.h and
 * include/siddhi_hip_ir.h alone (what a JNI or Panama binding sees): it builds the C1 program blob
 * by hand, creates an engine, pushes host batches and polls the R18-ordered matches.
 *
 *   c1_abi blob <path>           write the hand-built blob (tests/test_abi.py compares it with the
 *                                Python planner's serialization of the same query)
 *   c1_abi run <events> <batch>  run C1 over the seeded StockStream (siddhi_amd/workloads.py's
 *                                generator, restated below) and print "matches <n> hash <h>": h is an
 *                                FNV-1a over every delivered match's (query, key, ts, slot words) in
 *                                delivery order (tests/test_gpu_abi_c.py checks it against the oracle)
 *
 * C1 = BASELINE configs[0]: define stream StockStream (symbol string, price float, volume int);
 *      every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 10 sec
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "siddhi_hip.h"
#include "siddhi_hip_ir.h"

typedef struct {
  int64_t* w;
  size_t n, cap;
} Words;

static void put(Words* b, int64_t v) {
  if (b->n == b->cap) {
    b->cap = b->cap ? 2 * b->cap : 256;
    b->w = (int64_t*)realloc(b->w, b->cap * sizeof(int64_t));
  }
  b->w[b->n++] = v;
}

static void insn(Words* b, int op, int lt, int rt, int res, int64_t a, int64_t bb, int64_t imm) {
  put(b, SDH_INSN_W0(op, lt, rt, res));
  put(b, a);
  put(b, bb);
  put(b, imm);
}

/* one state record: kind stream is_start min max logical partner next_pre next_every_pre
 * within_every_pre callback_pre this_last_post has_selector waiting_ms */
static void state(Words* b, int is_start, int64_t next_pre, int64_t next_every_pre, int64_t within_every_pre,
                  int64_t this_last_post, int has_selector) {
  const int64_t v[14] = {SDH_K_STREAM, 0, is_start, 0, 0, 0, -1, next_pre, next_every_pre, within_every_pre,
                         -1, this_last_post, has_selector, -1};
  for (int i = 0; i < 14; ++i) put(b, v[i]);
}

/* the C1 program (siddhi_hip_ir.h grammar) */
static Words c1_blob(void) {
  Words b = {0};
  put(&b, SDH_IR_VERSION);
  put(&b, 1);                                          /* streams */
  put(&b, 3);                                          /*   StockStream (symbol, price, volume) */
  put(&b, SDH_T_STRING);
  put(&b, SDH_T_FLOAT);
  put(&b, SDH_T_INT);
  put(&b, 0);                                          /* strings */
  put(&b, 1);                                          /* queries */
  put(&b, SDH_Q_PATTERN);
  put(&b, 10000);                                      /*   within 10 sec */
  put(&b, 2);                                          /*   states e1, e2 */
  put(&b, -1);                                         /*   no partition */
  put(&b, 1);                                          /*   a selector */
  /* e1: the start state; `every` re-arms it (next_every_pre = within_every_pre = 0); its post feeds e2 */
  state(&b, 1, 1, 0, 0, 1, 0);
  put(&b, 1);                                          /*   filters: price > 20 */
  put(&b, 3);
  insn(&b, SDH_OP_ATTR, 0, 0, SDH_T_FLOAT, 0, SDH_IDX_CURRENT, 1);
  insn(&b, SDH_OP_CONST, 0, 0, SDH_T_INT, 0, 0, 20);
  insn(&b, SDH_OP_CMP, SDH_T_FLOAT, SDH_T_INT, SDH_T_BOOL, 0, 0, SDH_CMP_GT);
  /* e2: completes the match */
  state(&b, 0, -1, -1, -1, 1, 1);
  put(&b, 1);                                          /*   filters: price > e1.price */
  put(&b, 3);
  insn(&b, SDH_OP_ATTR, 0, 0, SDH_T_FLOAT, 1, SDH_IDX_CURRENT, 1);
  insn(&b, SDH_OP_ATTR, 0, 0, SDH_T_FLOAT, 0, SDH_IDX_CURRENT, 1);
  insn(&b, SDH_OP_CMP, SDH_T_FLOAT, SDH_T_FLOAT, SDH_T_BOOL, 0, 0, SDH_CMP_GT);
  put(&b, 1);                                          /*   start states */
  put(&b, 0);
  put(&b, 1);                                          /*   receivers: StockStream -> e1, e2 */
  put(&b, 0);
  put(&b, SDH_R_MULTI);
  put(&b, 2);
  put(&b, 0);
  put(&b, 1);
  put(&b, 4);                                          /*   runtime tree: next(every(e1), e2) */
  const int64_t nodes[16] = {SDH_N_NEXT, 2, 3, -1, SDH_N_STREAM, -1, -1, 0, SDH_N_EVERY, 1, -1, 0,
                             SDH_N_STREAM, -1, -1, 1};
  for (int i = 0; i < 16; ++i) put(&b, nodes[i]);
  put(&b, 2);                                          /*   outputs: e1.price as p1, e2.price as p2 */
  put(&b, 1);
  insn(&b, SDH_OP_ATTR, 0, 0, SDH_T_FLOAT, 0, 0, 1);
  put(&b, 1);
  insn(&b, SDH_OP_ATTR, 0, 0, SDH_T_FLOAT, 1, 0, 1);
  put(&b, 0);                                          /* partitions */
  return b;
}

static size_t blob_bytes(const Words* w, unsigned char** out) {
  const size_t n = 8 + w->n * 8;
  *out = (unsigned char*)malloc(n);
  memcpy(*out, SDH_IR_MAGIC, 8);
  memcpy(*out + 8, w->w, w->n * 8); /* (little-endian host) */
  return n;
}

/* siddhi_amd/workloads.py stock_events: h_j = splitmix64(seed ^ (4 i + j)) */
static uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void check(int rc, sdh_engine* e, const char* what) {
  if (rc != SDH_OK) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, sdh_last_error(e));
    exit(2);
  }
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: c1_abi blob <path> | c1_abi run <events> <batch>\n");
    return 1;
  }
  Words w = c1_blob();
  unsigned char* blob = NULL;
  const size_t len = blob_bytes(&w, &blob);
  if (!strcmp(argv[1], "blob")) {
    FILE* f = fopen(argv[2], "wb");
    if (!f || fwrite(blob, 1, len, f) != len) return 1;
    fclose(f);
    return 0;
  }
  const int64_t n = atoll(argv[2]), bs = argc > 3 ? atoll(argv[3]) : 4096;
  sdh_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = 0;
  cfg.shard_world = 1;
  cfg.partials_per_inst = 128;
  sdh_engine* e = NULL;
  check(sdh_engine_create(blob, len, &cfg, &e), NULL, "sdh_engine_create");
  int64_t* ts = (int64_t*)malloc(bs * 8);
  int32_t* sym = (int32_t*)malloc(bs * 4);
  float* price = (float*)malloc(bs * 4);
  int32_t* vol = (int32_t*)malloc(bs * 4);
  uint64_t h = 1469598103934665603ull, total = 0;
  for (int64_t lo = 0; lo < n; lo += bs) {
    const int64_t m = n - lo < bs ? n - lo : bs;
    for (int64_t k = 0; k < m; ++k) {
      const uint64_t i = (uint64_t)(lo + k);
      ts[k] = 1700000000000ll + (int64_t)i;
      price[k] = (float)(splitmix64(42ull ^ (4 * i + 1)) % 10000) / 100.0f;
      vol[k] = (int32_t)(1 + splitmix64(42ull ^ (4 * i + 2)) % 1000);
      sym[k] = (int32_t)(splitmix64(42ull ^ (4 * i + 3)) % 100);
    }
    const void* cols[3] = {sym, price, vol};
    sdh_batch b;
    memset(&b, 0, sizeof b);
    b.n = m;
    b.ts = ts;
    b.cols = cols;
    b.n_cols = 3;
    check(sdh_engine_push(e, 0, &b), e, "sdh_engine_push");
    sdh_matches out;
    check(sdh_engine_poll(e, &out), e, "sdh_engine_poll");
    for (int64_t i = 0; i < out.n; ++i) {
      const int64_t nw = out.off[i + 1] - out.off[i];
      const int64_t head[4] = {out.query[i], out.key[i], out.ts[i], nw};
      for (int j = 0; j < 4; ++j) h = (h ^ (uint64_t)head[j]) * 1099511628211ull;
      for (int64_t j = 0; j < nw; ++j) h = (h ^ (uint64_t)out.words[out.off[i] + j]) * 1099511628211ull;
    }
    total += (uint64_t)out.n;
  }
  sdh_engine_destroy(e);
  printf("matches %llu hash %llu\n", (unsigned long long)total, (unsigned long long)h);
  free(ts);
  free(sym);
  free(price);
  free(vol);
  free(blob);
  free(w.w);
  return 0;
}
