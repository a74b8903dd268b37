/*
 * synth.c -- seeded synthetic rating generator, libmfsynth.so.
 *
 * The reference ships no datasets (its only fixture is SparkExample.scala:54-104), so the
 * benchmark configs are synthetic with the shape of MovieLens / Netflix / Yahoo:
 *   items  ~ Zipf-Mandelbrot  p(i) ∝ (i + 1 + 80)^-1.0
 *   users  ~ Zipf-Mandelbrot  p(u) ∝ (u + 1 + 500)^-0.8
 *   rating = clip(round(3.6 + x_u . y_i + N(0, 0.5^2)), 1, 5), x, y ~ N(0, 0.25^2), rank 16
 *   ids 0-based, permuted with perm_seed; duplicates allowed; test split with split_seed.
 * Every value is a pure function of (seed, index), so the output does not depend on the
 * thread count and every rank of a multi-GPU job generates identical data.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t smix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
static inline double u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }
static inline double gauss(uint64_t a, uint64_t b) {
  double x = u01(a), y = u01(b);
  if (x < 1e-300) x = 1e-300;
  return sqrt(-2.0 * log(x)) * cos(6.283185307179586 * y);
}

static double* zipf_cdf(int64_t n, double q, double s) {
  double* c = (double*)malloc(sizeof(double) * (size_t)n);
  double acc = 0.0;
  for (int64_t x = 0; x < n; ++x) { acc += pow((double)x + 1.0 + q, -s); c[x] = acc; }
  for (int64_t x = 0; x < n; ++x) c[x] /= acc;
  c[n - 1] = 1.0;
  return c;
}
static inline int64_t draw(const double* cdf, int64_t n, double v) {
  int64_t lo = 0, hi = n - 1;
  while (lo < hi) { int64_t m = (lo + hi) >> 1; if (cdf[m] < v) lo = m + 1; else hi = m; }
  return lo;
}
static int32_t* permutation(int64_t n, uint64_t seed) {
  int32_t* p = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
  for (int64_t x = 0; x < n; ++x) p[x] = (int32_t)x;
  for (int64_t x = n - 1; x > 0; --x) {
    int64_t k = (int64_t)(smix(seed ^ smix((uint64_t)x)) % (uint64_t)(x + 1));
    int32_t t = p[x]; p[x] = p[k]; p[k] = t;
  }
  return p;
}

#define RANK 16
typedef struct {
  int64_t b, e, nu, ni;
  const double *cu, *ci;
  const float *X, *Y;
  const int32_t *pu, *pi;
  uint64_t seed, split_seed;
  double test_fraction;
  int32_t *u, *i;
  double* r;
  uint8_t* test;
} job;

static void* work(void* vp) {
  job* j = (job*)vp;
  for (int64_t x = j->b; x < j->e; ++x) {
    uint64_t h = smix(j->seed ^ smix((uint64_t)x * 4 + 1));
    int64_t ru = draw(j->cu, j->nu, u01(h));
    int64_t ri = draw(j->ci, j->ni, u01(smix(h ^ 0x1234567ULL)));
    const float* xu = j->X + ru * RANK;
    const float* yi = j->Y + ri * RANK;
    double dot = 0.0;
    for (int f = 0; f < RANK; ++f) dot += (double)xu[f] * (double)yi[f];
    double noise = 0.5 * gauss(smix(h ^ 0xABCDEFULL), smix(h ^ 0x7777ULL));
    double v = floor(3.6 + dot + noise + 0.5);
    if (v < 1.0) v = 1.0;
    if (v > 5.0) v = 5.0;
    j->u[x] = j->pu[ru];
    j->i[x] = j->pi[ri];
    j->r[x] = v;
    if (j->test) j->test[x] = u01(smix(j->split_seed ^ smix((uint64_t)x * 4 + 3))) < j->test_fraction;
  }
  return NULL;
}

/* Fills u, i, r (and test flags when test != NULL) for n ratings. */
int mfs_generate(int64_t n_users, int64_t n_items, int64_t n, uint64_t seed, uint64_t perm_seed,
                 uint64_t split_seed, double test_fraction, int threads, int32_t* u, int32_t* i,
                 double* r, uint8_t* test) {
  if (n_users < 1 || n_items < 1 || n < 0) return -1;
  double* cu = zipf_cdf(n_users, 500.0, 0.8);
  double* ci = zipf_cdf(n_items, 80.0, 1.0);
  float* X = (float*)malloc(sizeof(float) * (size_t)n_users * RANK);
  float* Y = (float*)malloc(sizeof(float) * (size_t)n_items * RANK);
  for (int64_t x = 0; x < n_users * RANK; ++x)
    X[x] = (float)(0.25 * gauss(smix(seed ^ smix((uint64_t)x * 2 + 11)), smix(seed ^ smix((uint64_t)x * 2 + 12))));
  for (int64_t x = 0; x < n_items * RANK; ++x)
    Y[x] = (float)(0.25 * gauss(smix(~seed ^ smix((uint64_t)x * 2 + 13)), smix(~seed ^ smix((uint64_t)x * 2 + 14))));
  int32_t* pu = permutation(n_users, perm_seed);
  int32_t* pi = permutation(n_items, perm_seed ^ 0x5555ULL);
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  job js[64];
  pthread_t th[64];
  int64_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    job* j = &js[t];
    j->b = t * chunk;
    j->e = j->b + chunk < n ? j->b + chunk : n;
    if (j->b > n) j->b = n;
    j->nu = n_users; j->ni = n_items; j->cu = cu; j->ci = ci; j->X = X; j->Y = Y; j->pu = pu; j->pi = pi;
    j->seed = seed; j->split_seed = split_seed; j->test_fraction = test_fraction;
    j->u = u; j->i = i; j->r = r; j->test = test;
    pthread_create(&th[t], NULL, work, j);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(cu); free(ci); free(X); free(Y); free(pu); free(pi);
  return 0;
}
