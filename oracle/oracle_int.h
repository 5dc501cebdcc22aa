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
#define ORC_FLAG_FUSED_ERROR 64   /* MCV_FLAG_FUSED_ERROR (bit 4 is retired) */
#define ORC_FLAG_CV_SAMPLER 32    /* MCV_FLAG_CV_SAMPLER */
#define ORC_FLAG_FAST_MINIMAL 16  /* MCV_FLAG_FAST_MINIMAL: the non-reference minimal solvers */
int orc_get_fast_minimal(void);
void orc_set_fast_minimal(int v);

/* Per-hypothesis word stream: word s = philox({s/4, hyp_lo, hyp_hi, "MCV1"}, {seed_lo, seed_hi})[s%4] */
typedef struct { uint64_t seed, hyp; uint64_t pos; uint32_t buf[4]; } Stream;

uint32_t stream_next(Stream* st);
int stream_uniform(Stream* st, int n);
int draw_distinct(Stream* st, int N, int m, int* idx);
int64_t orc_cv_subsets(int check, const float* pts4, int N, int m, int64_t rows, int* out);
int* orc_cv_begin(int flags, int check, const float* pts4, int N, int m, int64_t rows);
void orc_cv_end(int* t);
void jacobi3_orc(double* A, double* V);
float f_err_orc(int kind, const double* F, double x1, double y1, double x2, double y2);
int orc_update_num_iters(double p, double ep, int modelPoints, int maxIters);
int64_t orc_ransac_replay(const int* counts, int64_t ncounts, int N, int m, double conf, int maxIters, int fixed,
                          int* bestCount);
void eig_pinv_apply(const double* A, int n, const double* b, double* x, double* Ainv);
int orc_poly_real_roots(const double* cin, int deg, double* roots);
/* PnP (oracle_pnp.c / oracle_epnp.c) */
void orc_undistort(const double* cam8, double u, double v, double* x, double* y);
int orc_pnp_hypothesis(const float* pts, int N, const double* cam8, uint64_t seed, int64_t hyp, double* R, double* t,
                       int* idx_out);
int orc_pnp_count(const float* pts, int N, const double* cam8, const double* R, const double* t, float thr2, int fused,
                  uint8_t* mask);
void orc_pnp_lm(const float* pts, int N, const uint8_t* mask, const double* cam8, double* rvec, double* t,
                int maxIters);
void orc_rodrigues_inv(const double* R, double* r);
int orc_f_count(const float* pts4, int N, const double* F, float thr2, int kind, uint8_t* mask);
int64_t orc_ransac_replay_slots(const int* counts, int64_t nhyp, int slots, int N, int m, double conf, int maxIters,
                                int fixed, int* bestCount);
void orc_jsvd(double* At, double* Wout, double* Vt, int m, int n, int n1);
void orc_epnp(const double* pw, const double* us, int n, const double* cam4, double* R, double* t);
void orc_epnp5_f32(const float* p5, const double* cam8, double* R, double* t);
int orc_pnp_hypothesis_epnp(const float* pts, int N, const double* cam8, uint64_t seed, int64_t hyp, double* R,
                            double* t, int* idx_out);
void orc_epnp_points(const double* img, const double* world, int n, const double* cam8, double* R, double* t);
int orc_sqpnp(const double* img, const double* world, int n, const double* cam8, double* rvec, double* tvec);

#endif
