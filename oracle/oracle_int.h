/* oracle_int.h — helpers shared by the oracle's translation units (test infrastructure only). */
#ifndef ORACLE_INT_H
#define ORACLE_INT_H
#include <stdint.h>

#define ORC_MAX_ATTEMPTS 10000
#define ORC_MAX_REDRAW 1000
#define ORC_NO_MODEL (-1)
#define ORC_NO_SAMPLE (-2)

#define ORC_FLAG_FIXED_ITERS 1
#define ORC_FLAG_NO_REFINE 2
#define ORC_FLAG_FUSED_ERROR 4

/* Per-hypothesis word stream: word s = philox({s/4, hyp_lo, hyp_hi, "MCV1"}, {seed_lo, seed_hi})[s%4] */
typedef struct { uint64_t seed, hyp; uint64_t pos; uint32_t buf[4]; } Stream;

uint32_t stream_next(Stream* st);
int stream_uniform(Stream* st, int n);
int draw_distinct(Stream* st, int N, int m, int* idx);
void jacobi3_orc(double* A, double* V);
float f_err_orc(int kind, const double* F, double x1, double y1, double x2, double y2);
int orc_update_num_iters(double p, double ep, int modelPoints, int maxIters);
int64_t orc_ransac_replay(const int* counts, int64_t ncounts, int N, int m, double conf, int maxIters, int fixed,
                          int* bestCount);
void eig_pinv_apply(const double* A, int n, const double* b, double* x, double* Ainv);
int orc_poly_real_roots(const double* cin, int deg, double* roots);

#endif
