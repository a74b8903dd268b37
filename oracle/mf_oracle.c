/*
 * oracle/mf_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's DSGD / online-MF hot path, used as the
 * parity checker for the HIP product (libmfhip.so) and as the timed CPU baseline
 * ("cpu_baseline.kind" = "port") in bench.py.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product never links it.
 *
 * Parity pinning: the reference (Scala 2.11, Flink 1.3 / Spark 2.2) has no tests,
 * fixtures or golden outputs and cannot be built here (no JVM).  The JVM RNG and
 * Scala shuffle are pinned by JDK known-answer values (tests/test_oracle_rng.py);
 * the DSGD/online algorithms are a restatement of the cited reference lines and
 * are cross-checked against the independent Python restatement (oracle/mf_oracle.py).
 * Algorithm parity is therefore "unpinned beyond the RNG KATs" (see DESIGN.md).
 *
 * Reference paths (abbreviated as in SURVEY.md):
 *   fl/mf/offline/DSGDforMF.scala, fl/mf/offline/MatrixFactorization.scala,
 *   core/FactorUpdater.scala, core/FactorInitializer.scala,
 *   sp/OfflineSpark.scala, fl/mf/online/FlinkOnlineMF.scala
 *
 * Build: oracle/Makefile -> oracle/build/libmforacle.so  (gcc -O2 -ffp-contract=off)
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------- */
/* java.util.Random, JDK 8 specification (LCG 0x5DEECE66D, 48-bit state).     */
/* Used at DSGDforMF.scala:392,532,548 and core/FactorInitializer.scala:33.   */
/* ------------------------------------------------------------------------- */
typedef struct { uint64_t s; } jrand;
#define JR_MASK ((1ULL << 48) - 1)

static void jr_init(jrand* r, int64_t seed) { r->s = ((uint64_t)seed ^ 0x5DEECE66DULL) & JR_MASK; }

static int32_t jr_next(jrand* r, int bits) {
  r->s = (r->s * 0x5DEECE66DULL + 0xBULL) & JR_MASK;
  return (int32_t)(uint32_t)(r->s >> (48 - bits));
}

/* Random.nextInt(bound): power-of-two fast path, else rejection loop in int32. */
static int32_t jr_next_int_bound(jrand* r, int32_t bound) {
  int32_t x = jr_next(r, 31);
  int32_t m = bound - 1;
  if ((bound & m) == 0) return (int32_t)(((int64_t)bound * (int64_t)x) >> 31);
  for (int32_t u = x;; u = jr_next(r, 31)) {
    x = u % bound;
    if ((int32_t)((uint32_t)u - (uint32_t)x + (uint32_t)m) >= 0) break;
  }
  return x;
}

/* Random.nextDouble(): ((next(26) << 27) + next(27)) * 2^-53 */
static double jr_next_double(jrand* r) {
  int64_t hi = (int64_t)jr_next(r, 26);
  int64_t lo = (int64_t)jr_next(r, 27);
  return (double)((hi << 27) + lo) * (1.0 / 9007199254740992.0);
}

/* scala.util.Random.shuffle (Scala 2.11): for n = len..2 { k = nextInt(n); swap(n-1, k) } */
static void scala_shuffle_indices(jrand* r, int32_t* buf, int64_t len) {
  for (int64_t i = 0; i < len; ++i) buf[i] = (int32_t)i;
  for (int64_t n = len; n >= 2; --n) {
    int32_t k = jr_next_int_bound(r, (int32_t)n);
    int32_t t = buf[n - 1];
    buf[n - 1] = buf[k];
    buf[k] = t;
  }
}

/* ---- exported RNG helpers (known-answer tests) ---- */
void orc_jr_next_int(int64_t seed, int32_t count, int32_t* out) {
  jrand r; jr_init(&r, seed);
  for (int32_t j = 0; j < count; ++j) out[j] = jr_next(&r, 32);
}
void orc_jr_next_int_bound(int64_t seed, int32_t bound, int32_t count, int32_t* out) {
  jrand r; jr_init(&r, seed);
  for (int32_t j = 0; j < count; ++j) out[j] = jr_next_int_bound(&r, bound);
}
void orc_jr_next_double(int64_t seed, int32_t count, double* out) {
  jrand r; jr_init(&r, seed);
  for (int32_t j = 0; j < count; ++j) out[j] = jr_next_double(&r);
}
void orc_scala_shuffle(int64_t seed, int64_t len, int32_t* out) {
  jrand r; jr_init(&r, seed);
  scala_shuffle_indices(&r, out, len);
}
/* DSGDforMF.scala:531-533: new Random(id ^ seed).nextInt(numBlocks); id is Int, sign-extended. */
int32_t orc_block_of(int32_t id, int64_t seed, int32_t n_blocks) {
  jrand r; jr_init(&r, (int64_t)id ^ seed);
  return jr_next_int_bound(&r, n_blocks);
}
/* MatrixFactorization.scala:278-280 with DSGDforMF.scala:548 (fresh Random(id ^ seed)). */
void orc_random_factors(int64_t rng_seed, int32_t k, double* out) {
  jrand r; jr_init(&r, rng_seed);
  for (int32_t f = 0; f < k; ++f) out[f] = jr_next_double(&r);
}

/* ------------------------------------------------------------------------- */
/* flink-ml 1.3.0 LearningRateMethod (restated; DSGDforMF.scala:10,383-386).  */
/* ------------------------------------------------------------------------- */
enum { LR_DEFAULT = 0, LR_CONSTANT = 1, LR_BOTTOU = 2, LR_INVSCALING = 3, LR_XU = 4 };
double orc_learning_rate(int method, double lr, int32_t iteration, double lambda, double arg) {
  switch (method) {
    case LR_CONSTANT: return lr;
    case LR_BOTTOU: return 1.0 / (lambda * (arg + (double)iteration - 1.0));
    case LR_INVSCALING: return lr / pow((double)iteration, arg);
    case LR_XU: return lr * pow(1.0 + lambda * lr * (double)iteration, -arg);
    default: return lr / sqrt((double)iteration);
  }
}

/* ------------------------------------------------------------------------- */
/* The per-rating DSGD update, DSGDforMF.scala:395-414 (exact JVM order).     */
/* ------------------------------------------------------------------------- */
static void dsgd_update(double* p, double* q, int32_t k, double r, double eta,
                        double reg_u, double reg_i) {
  /* netlib-java F2jBLAS.ddot: sequential left fold from 0.0 (its unroll-by-5 body
     is written ((((dtemp + x0*y0) + x1*y1) + ...), so the order is unchanged). */
  double dot = 0.0;
  for (int32_t f = 0; f < k; ++f) dot = dot + p[f] * q[f];
  double e = r - dot;                                    /* :405 piqj */
  for (int32_t f = 0; f < k; ++f) {
    double pf = p[f], qf = q[f];
    double np = pf - eta * (reg_u * pf - e * qf);        /* :407-408 (lambda/omega_i)*p */
    double nq = qf - eta * (reg_i * qf - e * pf);        /* :409-410 uses the old p */
    p[f] = np;
    q[f] = nq;
  }
}

/* Exact updateLocalFactors replacement on caller buffers (DSGDforMF.scala:378-418):
   users/items are row-major [rows x k] factor slabs of the two blocks. */
void orc_block_update(const double* r, const int32_t* uidx, const int32_t* iidx, int64_t len,
                      double* users, const int32_t* uomega, double* items, const int32_t* iomega,
                      int32_t k, int32_t iteration, int32_t rating_block_id, int64_t seed,
                      double lr, int32_t lr_method, double lr_arg, double lambda) {
  double eta = orc_learning_rate(lr_method, lr, iteration + 1, lambda, lr_arg);
  int32_t* order = (int32_t*)malloc(sizeof(int32_t) * (size_t)(len > 0 ? len : 1));
  jrand rng; jr_init(&rng, (int64_t)(iteration ^ rating_block_id) ^ seed);
  scala_shuffle_indices(&rng, order, len);
  for (int64_t j = 0; j < len; ++j) {
    int32_t x = order[j];
    int32_t ur = uidx[x], ir = iidx[x];
    dsgd_update(users + (size_t)ur * k, items + (size_t)ir * k, k, r[x], eta,
                lambda / (double)uomega[ur], lambda / (double)iomega[ir]);
  }
  free(order);
}

/* ------------------------------------------------------------------------- */
/* Stable LSD radix sort of (key64, idx32).                                   */
/* ------------------------------------------------------------------------- */
static void radix_sort64(uint64_t* key, int32_t* idx, int64_t n, int key_bits) {
  uint64_t* k2 = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(n ? n : 1));
  int32_t* i2 = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  int64_t* cnt = (int64_t*)malloc(sizeof(int64_t) * 65536);
  for (int shift = 0; shift < key_bits; shift += 16) {
    memset(cnt, 0, sizeof(int64_t) * 65536);
    for (int64_t j = 0; j < n; ++j) cnt[(key[j] >> shift) & 0xFFFF]++;
    int64_t acc = 0;
    for (int d = 0; d < 65536; ++d) { int64_t c = cnt[d]; cnt[d] = acc; acc += c; }
    for (int64_t j = 0; j < n; ++j) {
      int64_t pos = cnt[(key[j] >> shift) & 0xFFFF]++;
      k2[pos] = key[j];
      i2[pos] = idx[j];
    }
    memcpy(key, k2, sizeof(uint64_t) * (size_t)n);
    memcpy(idx, i2, sizeof(int32_t) * (size_t)n);
  }
  free(k2); free(i2); free(cnt);
}

static inline uint32_t flip(int32_t x) { return (uint32_t)x ^ 0x80000000u; }

/* Distinct ids (ascending, signed order) with occurrence counts. */
typedef struct {
  int64_t count;
  int32_t* ids;     /* sorted distinct ids          */
  int32_t* omega;   /* ratings per id (:537-541)    */
  int32_t* block;   /* factor block id (:531-533)   */
  int64_t* row;     /* global row = block_start + idx_in_block (ids sorted in a block, :556) */
  int64_t* block_start; /* n_blocks + 1 */
} side_index;

static void side_build(side_index* s, const int32_t* ids, int64_t n, int32_t n_blocks, int64_t seed) {
  uint64_t* key = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(n ? n : 1));
  int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  for (int64_t j = 0; j < n; ++j) { key[j] = flip(ids[j]); idx[j] = (int32_t)j; }
  radix_sort64(key, idx, n, 32);
  int64_t d = 0;
  for (int64_t j = 0; j < n; ++j) if (j == 0 || key[j] != key[j - 1]) d++;
  s->count = d;
  s->ids = (int32_t*)malloc(sizeof(int32_t) * (size_t)(d ? d : 1));
  s->omega = (int32_t*)calloc((size_t)(d ? d : 1), sizeof(int32_t));
  s->block = (int32_t*)malloc(sizeof(int32_t) * (size_t)(d ? d : 1));
  s->row = (int64_t*)malloc(sizeof(int64_t) * (size_t)(d ? d : 1));
  s->block_start = (int64_t*)calloc((size_t)n_blocks + 1, sizeof(int64_t));
  int64_t c = -1;
  for (int64_t j = 0; j < n; ++j) {
    if (j == 0 || key[j] != key[j - 1]) { c++; s->ids[c] = (int32_t)(key[j] ^ 0x80000000u); }
    s->omega[c]++;
  }
  for (int64_t x = 0; x < d; ++x) {
    s->block[x] = orc_block_of(s->ids[x], seed, n_blocks);
    s->block_start[s->block[x] + 1]++;
  }
  for (int32_t b = 0; b < n_blocks; ++b) s->block_start[b + 1] += s->block_start[b];
  int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)n_blocks);
  for (int32_t b = 0; b < n_blocks; ++b) fill[b] = s->block_start[b];
  for (int64_t x = 0; x < d; ++x) s->row[x] = fill[s->block[x]]++;  /* ascending ids => sorted in block */
  free(fill); free(key); free(idx);
}

static int64_t side_find(const side_index* s, int32_t id) {
  int64_t lo = 0, hi = s->count - 1;
  while (lo <= hi) {
    int64_t mid = (lo + hi) >> 1;
    if (s->ids[mid] == id) return mid;
    if (s->ids[mid] < id) lo = mid + 1; else hi = mid - 1;
  }
  return -1;
}

static void side_free(side_index* s) {
  free(s->ids); free(s->omega); free(s->block); free(s->row); free(s->block_start);
}

/* ------------------------------------------------------------------------- */
/* DSGD fit (DSGDforMF.fitSGD, :262-357).                                     */
/* ------------------------------------------------------------------------- */
typedef struct orc_model {
  int32_t k;
  side_index su, si;
  double* uf;   /* [users x k] by global row */
  double* itf;  /* [items x k] by global row */
  /* rating blocks */
  int32_t n_blocks;
  int64_t* rb_start;   /* n*n + 1 */
  int32_t* rb_urow;    /* row index within the user block */
  int32_t* rb_irow;    /* row index within the item block */
  double* rb_r;
  double* reg_u;       /* lambda / omega per global row */
  double* reg_i;
} orc_model;

typedef struct {
  orc_model* m;
  int32_t tid, nthreads, superstep, iteration;
  int64_t seed;
  double eta;
  int64_t updates;
} sweep_arg;

/* updateFactors (:364-497) for one superstep: rating block (p, (p+s-1) mod n) for every p. */
static void* sweep_worker(void* vp) {
  sweep_arg* a = (sweep_arg*)vp;
  orc_model* m = a->m;
  int32_t n = m->n_blocks, k = m->k;
  for (int32_t p = a->tid; p < n; p += a->nthreads) {
    int32_t q = (p + a->superstep - 1) % n;
    int32_t rbid = p * n + q;                       /* toRatingBlockId :597-601 */
    int64_t s0 = m->rb_start[rbid], len = m->rb_start[rbid + 1] - s0;
    if (len == 0) continue;                         /* empty rating block passes through :482-487 */
    double* users = m->uf + (size_t)m->su.block_start[p] * k;
    double* items = m->itf + (size_t)m->si.block_start[q] * k;
    const double* ru = m->reg_u + m->su.block_start[p];
    const double* ri = m->reg_i + m->si.block_start[q];
    int32_t* order = (int32_t*)malloc(sizeof(int32_t) * (size_t)len);
    jrand rng; jr_init(&rng, (int64_t)(a->iteration ^ rbid) ^ a->seed);   /* :392 */
    scala_shuffle_indices(&rng, order, len);                              /* :393 */
    for (int64_t j = 0; j < len; ++j) {
      int64_t x = s0 + order[j];
      int32_t ur = m->rb_urow[x], ir = m->rb_irow[x];
      dsgd_update(users + (size_t)ur * k, items + (size_t)ir * k, k, m->rb_r[x], a->eta, ru[ur], ri[ir]);
    }
    a->updates += len;
    free(order);
  }
  return NULL;
}

static double now_s(void) {
  struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

orc_model* orc_dsgd_fit(int32_t k, int32_t iterations, double lambda, double lr, int32_t lr_method,
                        double lr_arg, int32_t n_blocks, int64_t seed, int32_t threads,
                        int64_t max_supersteps, const int32_t* u, const int32_t* i, const double* r,
                        int64_t n, double* sweep_seconds, int64_t* updates_done) {
  if (n_blocks < 1) n_blocks = 1;
  orc_model* m = (orc_model*)calloc(1, sizeof(orc_model));
  m->k = k;
  m->n_blocks = n_blocks;
  side_build(&m->su, u, n, n_blocks, seed);   /* initFactorBlockAndIndices(users) :286-287 */
  side_build(&m->si, i, n, n_blocks, seed);   /* initFactorBlockAndIndices(items) :288-289 */
  int64_t U = m->su.count, I = m->si.count;
  m->uf = (double*)malloc(sizeof(double) * (size_t)(U ? U : 1) * k);
  m->itf = (double*)malloc(sizeof(double) * (size_t)(I ? I : 1) * k);
  m->reg_u = (double*)malloc(sizeof(double) * (size_t)(U ? U : 1));
  m->reg_i = (double*)malloc(sizeof(double) * (size_t)(I ? I : 1));
  for (int64_t x = 0; x < U; ++x) {
    orc_random_factors((int64_t)m->su.ids[x] ^ seed, k, m->uf + (size_t)m->su.row[x] * k);  /* :548-549 */
    m->reg_u[m->su.row[x]] = lambda / (double)m->su.omega[x];
  }
  for (int64_t x = 0; x < I; ++x) {
    orc_random_factors((int64_t)m->si.ids[x] ^ seed, k, m->itf + (size_t)m->si.row[x] * k);
    m->reg_i[m->si.row[x]] = lambda / (double)m->si.omega[x];
  }
  /* Rating blocks (:301-327): block = ub*n + ib; sorted by (user, item), stable. */
  uint64_t* key = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(n ? n : 1));
  int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  int64_t* ux = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n ? n : 1));
  int64_t* ix = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n ? n : 1));
  for (int64_t j = 0; j < n; ++j) {
    key[j] = ((uint64_t)flip(u[j]) << 32) | flip(i[j]);
    idx[j] = (int32_t)j;
    ux[j] = side_find(&m->su, u[j]);
    ix[j] = side_find(&m->si, i[j]);
  }
  radix_sort64(key, idx, n, 64);
  int64_t nb2 = (int64_t)n_blocks * n_blocks;
  m->rb_start = (int64_t*)calloc((size_t)nb2 + 1, sizeof(int64_t));
  for (int64_t j = 0; j < n; ++j)
    m->rb_start[(int64_t)m->su.block[ux[j]] * n_blocks + m->si.block[ix[j]] + 1]++;
  for (int64_t b = 0; b < nb2; ++b) m->rb_start[b + 1] += m->rb_start[b];
  int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)nb2);
  for (int64_t b = 0; b < nb2; ++b) fill[b] = m->rb_start[b];
  m->rb_urow = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  m->rb_irow = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  m->rb_r = (double*)malloc(sizeof(double) * (size_t)(n ? n : 1));
  for (int64_t j = 0; j < n; ++j) {   /* counting sort by block over the (u,i)-sorted order: stable */
    int32_t src = idx[j];
    int64_t xu = ux[src], xi = ix[src];
    int32_t ub = m->su.block[xu], ib = m->si.block[xi];
    int64_t pos = fill[(int64_t)ub * n_blocks + ib]++;
    m->rb_urow[pos] = (int32_t)(m->su.row[xu] - m->su.block_start[ub]);
    m->rb_irow[pos] = (int32_t)(m->si.row[xi] - m->si.block_start[ib]);
    m->rb_r[pos] = r[src];
  }
  free(fill); free(key); free(idx); free(ux); free(ix);

  /* BulkIteration: iterations * numBlocks supersteps (:341-344), superstep is 1-based. */
  int64_t total = (int64_t)iterations * n_blocks;
  if (max_supersteps >= 0 && max_supersteps < total) total = max_supersteps;
  if (threads < 1) threads = 1;
  if (threads > n_blocks) threads = n_blocks;
  sweep_arg* args = (sweep_arg*)calloc((size_t)threads, sizeof(sweep_arg));
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
  int64_t updates = 0;
  double t0 = now_s();
  for (int64_t s = 1; s <= total; ++s) {
    int32_t iteration = (int32_t)(s / n_blocks);                         /* :476 */
    double eta = orc_learning_rate(lr_method, lr, iteration + 1, lambda, lr_arg);   /* :383-386 */
    for (int32_t t = 0; t < threads; ++t) {
      args[t].m = m; args[t].tid = t; args[t].nthreads = threads;
      args[t].superstep = (int32_t)s; args[t].iteration = iteration;
      args[t].seed = seed; args[t].eta = eta; args[t].updates = 0;
    }
    if (threads == 1) sweep_worker(&args[0]);
    else {
      for (int32_t t = 0; t < threads; ++t) pthread_create(&th[t], NULL, sweep_worker, &args[t]);
      for (int32_t t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    }
    for (int32_t t = 0; t < threads; ++t) updates += args[t].updates;
  }
  double t1 = now_s();
  if (sweep_seconds) *sweep_seconds = t1 - t0;
  if (updates_done) *updates_done = updates;
  free(args); free(th);
  return m;
}

int64_t orc_model_count(const orc_model* m, int32_t side) { return side == 0 ? m->su.count : m->si.count; }

/* unblock (:245-255): (id, factors) for every id; returned in ascending id order. */
void orc_model_get(const orc_model* m, int32_t side, int32_t* ids, double* vecs) {
  const side_index* s = side == 0 ? &m->su : &m->si;
  const double* f = side == 0 ? m->uf : m->itf;
  for (int64_t x = 0; x < s->count; ++x) {
    ids[x] = s->ids[x];
    memcpy(vecs + (size_t)x * m->k, f + (size_t)s->row[x] * m->k, sizeof(double) * (size_t)m->k);
  }
}

/* predictRating (MatrixFactorization.scala:239-274): inner join, then ddot. */
void orc_model_predict(const orc_model* m, const int32_t* u, const int32_t* i, int64_t n,
                       double* out, uint8_t* found) {
  for (int64_t j = 0; j < n; ++j) {
    int64_t xu = side_find(&m->su, u[j]), xi = side_find(&m->si, i[j]);
    if (xu < 0 || xi < 0) { found[j] = 0; out[j] = 0.0; continue; }
    const double* p = m->uf + (size_t)m->su.row[xu] * m->k;
    const double* q = m->itf + (size_t)m->si.row[xi] * m->k;
    double dot = 0.0;
    for (int32_t f = 0; f < m->k; ++f) dot = dot + p[f] * q[f];
    found[j] = 1;
    out[j] = dot;
  }
}

void orc_model_free(orc_model* m) {
  if (!m) return;
  side_free(&m->su); side_free(&m->si);
  free(m->uf); free(m->itf); free(m->reg_u); free(m->reg_i);
  free(m->rb_start); free(m->rb_urow); free(m->rb_irow); free(m->rb_r);
  free(m);
}

/* ------------------------------------------------------------------------- */
/* Online MF: SGDUpdater.nextFactors (core/FactorUpdater.scala:35-45) applied  */
/* in a caller-given sequential order on a dense model (rows = caller slots).  */
/* The caller resolves ids -> rows and initialises unseen rows               */
/* (PseudoRandomFactorInitializer, core/FactorInitializer.scala:23-27).      */
/* ------------------------------------------------------------------------- */
void orc_online_apply(const int32_t* urow, const int32_t* irow, const double* r, int64_t n,
                      double* users, double* items, int32_t k, double lr) {
  for (int64_t j = 0; j < n; ++j) {
    double* p = users + (size_t)urow[j] * k;
    double* q = items + (size_t)irow[j] * k;
    double dot = 0.0;                              /* zip.map(x*y).sum: foldLeft from 0.0 */
    for (int32_t f = 0; f < k; ++f) dot = dot + p[f] * q[f];
    double e = r[j] - dot;
    double le = lr * e;                            /* learningRate * e * i == (lr*e)*i */
    for (int32_t f = 0; f < k; ++f) {
      double pf = p[f], qf = q[f];
      p[f] = pf + le * qf;
      q[f] = qf + le * pf;
    }
  }
}

/* Sequential DSGD updates (DSGDforMF.scala:405-413) over caller rows in the given order with a
   fixed learning rate: replays a schedule serialised by the caller (e.g. the fast-mode plan). */
void orc_dsgd_apply(const int32_t* urow, const int32_t* irow, const double* r, int64_t n,
                    double* users, double* items, const double* reg_u, const double* reg_i,
                    int32_t k, double eta) {
  for (int64_t j = 0; j < n; ++j)
    dsgd_update(users + (size_t)urow[j] * k, items + (size_t)irow[j] * k, k, r[j], eta,
                reg_u[urow[j]], reg_i[irow[j]]);
}
