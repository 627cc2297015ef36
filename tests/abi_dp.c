/*
 * abi_dp.c — a plain-C caller of the drop-in host library's data-parallel
 * path (include/rram_caffe.h rram_comm_* / rram_dp_*), the shape of the
 * reference's `caffe train -gpu 0,1,...` (tools/caffe.cpp:247-249:
 * P2PSync<float> sync(solver, NULL, param); sync.Run(gpus)) for one process
 * per GPU.  Built by rram-caffe-simulation_amd/Makefile into build/abi_dp;
 * tests/test_gpu_native_dp.py runs it.
 *
 *   abi_dp SOLVER.prototxt NET.prototxt OPTIONS ITERS OUT.bin [RANK WORLD ID_FILE [OVERLAP]]
 *
 * Rank r selects device (r mod device count), rank 0 draws the RCCL id and
 * writes it to ID_FILE for the other ranks (world 1: no file).  Trains ITERS
 * iterations with the gradients all-reduced by the library's P2PSync, then
 * rank 0 writes the flat parameter buffer (float32) followed by the broken
 * cell counts (uint64) to OUT.bin and prints one summary line.
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "rram_caffe.h"

#define CK(x)                                                                          \
  do {                                                                                 \
    int rc_ = (x);                                                                     \
    if (rc_ != 0) {                                                                    \
      fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #x, rc_, rram_caffe_last_error()); \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

static char* slurp(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  char* s = (char*)malloc((size_t)n + 1);
  if (s && fread(s, 1, (size_t)n, f) != (size_t)n) {
    free(s);
    s = NULL;
  }
  if (s) s[n] = 0;
  fclose(f);
  return s;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s SOLVER NET OPTIONS ITERS OUT [RANK WORLD ID_FILE [OVERLAP]]\n", argv[0]);
    return 2;
  }
  const int iters = atoi(argv[4]);
  const int rank = argc > 6 ? atoi(argv[6]) : 0;
  const int world = argc > 7 ? atoi(argv[7]) : 1;
  const char* id_file = argc > 8 ? argv[8] : NULL;
  const int overlap = argc > 9 ? atoi(argv[9]) : 1;
  char* solver_txt = slurp(argv[1]);
  char* net_txt = slurp(argv[2]);
  if (!solver_txt || !net_txt) {
    fprintf(stderr, "cannot read %s / %s\n", argv[1], argv[2]);
    return 2;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
    fprintf(stderr, "no GPU\n");
    return 3;
  }
  if (hipSetDevice(rank % ndev) != hipSuccess) return 3;

  /* every rank: identical seed (same weights and fault maps), its own data shard */
  char opts[4096];
  snprintf(opts, sizeof opts, "%s data_seed: %d", argv[3], rank);
  CK(rram_caffe_set_stream(NULL));
  CK(rram_caffe_set_random_seed(1701));
  rram_solver_t s = NULL;
  CK(rram_solver_create(solver_txt, net_txt, opts, &s));

  unsigned char id[RRAM_COMM_ID_BYTES];
  if (rank == 0) {
    CK(rram_comm_unique_id(id));
    if (world > 1) {
      char tmp[4096];
      snprintf(tmp, sizeof tmp, "%s.tmp", id_file);
      FILE* f = fopen(tmp, "wb");
      if (!f || fwrite(id, 1, sizeof id, f) != sizeof id) return 4;
      fclose(f);
      rename(tmp, id_file); /* atomic publish */
    }
  } else {
    FILE* f = NULL;
    for (int t = 0; t < 6000 && !f; ++t) { /* up to 60 s */
      f = fopen(id_file, "rb");
      if (!f) usleep(10000);
    }
    if (!f || fread(id, 1, sizeof id, f) != sizeof id) return 4;
    fclose(f);
  }
  rram_comm_t c = NULL;
  CK(rram_comm_create(id, rank, world, &c));
  rram_dp_t dp = NULL;
  CK(rram_dp_create(s, c, 4.0, overlap, &dp));
  CK(rram_solver_step(s, iters));
  CK(rram_caffe_synchronize());

  long long calls = 0, bcalls = 0;
  int buckets = 0;
  int64_t n = 0;
  CK(rram_dp_info(dp, &calls, &bcalls, &buckets, &n));
  float *data = NULL, *diff = NULL;
  int64_t nf = 0;
  CK(rram_solver_flat_params(s, &data, &diff, &nf));
  unsigned long long broken[256];
  int nb = 0;
  CK(rram_solver_broken_counts(s, broken, 256, &nb));
  if (rank == 0) {
    float* h = (float*)malloc((size_t)nf * sizeof(float));
    if (!h || hipMemcpy(h, data, (size_t)nf * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) return 5;
    FILE* f = fopen(argv[5], "wb");
    if (!f) return 5;
    fwrite(h, sizeof(float), (size_t)nf, f);
    fwrite(broken, sizeof(unsigned long long), (size_t)nb, f);
    fclose(f);
    free(h);
    int r = 0, w = 0;
    CK(rram_comm_info(c, &r, &w));
    printf("abi_dp rank %d world %d iters %d params %lld allreduce_calls %lld bucket_calls %lld buckets %d "
           "fault_blobs %d\n",
           r, w, iters, (long long)n, calls, bcalls, buckets, nb);
  }
  CK(rram_dp_destroy(dp));
  CK(rram_comm_destroy(c));
  CK(rram_solver_destroy(s));
  free(solver_txt);
  free(net_txt);
  return 0;
}
