/*
 * mfhip.h -- C ABI of libmfhip.so, the MI355X-native DSGD / online-MF hot path.
 *
 * The reference (Mallik-G/large-scale-recommendation, Scala 2.11) runs this path on
 * Flink/Spark; a Scala shim binds these entry points over JNI.
 * Each entry point names the reference interface it replaces (file:line, paths as in
 * fl/mf = flink-adaptive-recom/src/main/scala/hu/sztaki/ilab/mf,
 * core = core/src/main/scala/hu/sztaki/ilab/recom/core,
 * sp = spark-adaptive-recom/src/main/scala/hu/sztaki/ilab/recom/spark).
 *
 * Conventions
 *  - Every call returns an int status: MF_OK (0) or a negative MF_ERR_*.
 *    mf_last_error() returns a thread-local message for the last failing call.
 *    The JNI shim maps a non-zero status to RuntimeException, like the reference
 *    (fl/mf/offline/MatrixFactorization.scala:189-190, 270-271).
 *  - Host buffers are caller-owned and never retained past the call.  Device state
 *    (factor slabs, rating blocks, schedules) is owned by the mf_ctx.
 *  - One mf_ctx is not thread-safe; distinct contexts are.
 *  - Ids are the reference's Int ids (user / item id spaces are separate).
 *  - Factor vectors cross the boundary as row-major double[count * k] (the JVM's
 *    Array[Double]); FAST_F32 mode stores f32 on the device and widens on the way out.
 */
#ifndef MFHIP_H
#define MFHIP_H

#include <stdint.h>

/* Testing hooks (schedule and ring invariants, plan digests) are declared in mfhip_testing.h:
   exported by the same library for the test suite, not part of the product surface. */

#ifdef __cplusplus
extern "C" {
#endif

#define MF_OK 0
#define MF_ERR_INVALID (-1)      /* bad argument (IllegalArgumentException)          */
#define MF_ERR_HIP (-2)          /* HIP runtime error                                */
#define MF_ERR_NOT_FITTED (-3)   /* predict before fit (MatrixFactorization.scala:270) */
#define MF_ERR_NO_DEVICE (-4)    /* no usable GPU: the library never falls back to CPU */
#define MF_ERR_COMM (-5)         /* RCCL error                                       */
#define MF_ERR_CAPACITY (-6)     /* caller buffer too small                          */
#define MF_ERR_STATE (-7)        /* call out of order                                */
#define MF_ERR_TIMEOUT (-8)      /* a device-side bound tripped                      */

/* Update arithmetic / precision. */
#define MF_MODE_DETERMINISTIC_F64 0 /* bitwise replay of the reference's update order  */
#define MF_MODE_FAST_F32 1          /* conflict-free rotation schedule, f32 factors    */

/* flink-ml 1.3 LearningRateMethod (fl/mf/offline/DSGDforMF.scala:10,167-169). */
#define MF_LR_DEFAULT 0    /* lr / sqrt(t)                              */
#define MF_LR_CONSTANT 1   /* lr                                        */
#define MF_LR_BOTTOU 2     /* 1 / (lambda * (lr_arg + t - 1))           */
#define MF_LR_INVSCALING 3 /* lr / t^lr_arg                             */
#define MF_LR_XU 4         /* lr * (1 + lambda*lr*t)^-lr_arg            */

/* Factor sides. */
#define MF_SIDE_USER 0
#define MF_SIDE_ITEM 1

/* Online update flavours (core/FactorUpdater.scala; sp/OfflineSpark.scala). */
#define MF_ONLINE_NEXT_FACTORS 0 /* SGDUpdater.nextFactors, ratings in arrival order    */
#define MF_ONLINE_DELTA 1        /* SGDUpdater.delta + "vec + delta" (PS path)          */
#define MF_ONLINE_SPARK_SWEEP 2  /* OfflineSpark.offlineDSGDUpdatesOnly order           */

/* Fast-mode factor blocking (DSGDforMF.scala:531-533 is the reference's). */
#define MF_BLOCKING_REFERENCE 0  /* new Random(id ^ seed).nextInt(numBlocks) (default)   */
#define MF_BLOCKING_BALANCED 1   /* rating-count balanced blocks (faster; different RMSE) */

/* Initialisers for ids first seen online (core/FactorInitializer.scala). */
#define MF_INIT_PSEUDO_RANDOM 0  /* new Random(id), k x nextDouble   (:23-27)           */
#define MF_INIT_SEEDED 1         /* new Random(id ^ seed), as DSGD init (DSGDforMF.scala:548) */

#define MF_UID_BYTES 128         /* RCCL unique id */

/* Parameters mirror MatrixFactorization.scala:201-223 and DSGDforMF.scala:163-169;
   mf_params_init fills the reference defaults. */
typedef struct mf_params {
  int32_t num_factors;     /* NumFactors, default 10                                  */
  int32_t iterations;      /* Iterations, default 10                                  */
  double lambda;           /* Lambda, default 1.0                                     */
  double learning_rate;    /* LearningRate, default 0.001                             */
  int32_t lr_method;       /* MF_LR_*, default MF_LR_DEFAULT                          */
  double lr_arg;           /* Bottou optimalInit / InvScaling,Xu decay                */
  int32_t num_blocks;      /* Blocks, default None -> 1                               */
  int64_t seed;            /* Seed, default Some(0)                                   */
  int32_t has_seed;        /* 1 = Some(seed) (deterministic), 0 = None                */
  int32_t mode;            /* MF_MODE_*, default MF_MODE_DETERMINISTIC_F64            */
  /* online path (core/FactorUpdater.scala:35-54, FactorInitializer.scala) */
  double online_learning_rate; /* SGDUpdater(learningRate), default 0.01               */
  int32_t online_init;         /* MF_INIT_*, default MF_INIT_PSEUDO_RANDOM              */
  /* fast-mode tuning: waves per device for the rotation schedule (0 = auto);
     a negative value -G fixes G rotation groups per rating block */
  int32_t fast_waves;
  /* fast-mode blocking: MF_BLOCKING_REFERENCE (default) or MF_BLOCKING_BALANCED;
     the deterministic mode always uses the reference's blocking */
  int32_t fast_blocking;
  int32_t reserved[6];
} mf_params;

/* Aggregated device statistics (timed with HIP events on the library's stream). */
typedef struct mf_stats {
  int64_t updates;           /* rating updates executed                          */
  int64_t supersteps;        /* DSGD supersteps executed                         */
  int64_t kernel_launches;   /* launches of the dominant (sweep) kernel          */
  double kernel_ms;          /* summed device time of those launches (profiling on) */
  double algorithmic_bytes;  /* updates x B(k) (16k+20 f32, 32k+24 f64)          */
  int64_t levels;            /* deterministic mode: dependency levels launched   */
  int32_t groups;            /* fast mode: rotation groups per rating block      */
  int32_t reserved0;
  int64_t pads;              /* fast mode: no-op records the plan inserted       */
  double moved_bytes;        /* bytes the sweep kernels request from memory: every row load and
                                store they issue (forwarded rows and no-op halves excluded) plus
                                the schedule records they read; an upper bound on HBM traffic */
} mf_stats;

typedef struct mf_ctx mf_ctx;

void mf_params_init(mf_params* p);
const char* mf_last_error(void);
const char* mf_version(void);
int mf_device_count(int* n);

/* Context on n_devices GPUs of this process (device_ids may be NULL -> 0..n-1). */
int mf_create(const mf_params* p, const int* device_ids, int n_devices, mf_ctx** out);
/* Context for one rank of a multi-process job (one process per GPU, RCCL over xGMI).
   uid comes from mf_comm_unique_id on rank 0, shipped to all ranks by the caller. */
int mf_comm_unique_id(uint8_t uid_out[MF_UID_BYTES]);
int mf_create_rank(const mf_params* p, int device_id, int nranks, int rank,
                   const uint8_t uid[MF_UID_BYTES], mf_ctx** out);
int mf_destroy(mf_ctx* ctx);

/* DSGDforMF.fitSGD.fit (fl/mf/offline/DSGDforMF.scala:262-357): blocking, all
   iterations*numBlocks supersteps and unblocking.  Copies the caller's arrays. */
int mf_dsgd_fit(mf_ctx* ctx, const int32_t* users, const int32_t* items, const double* ratings,
                int64_t n);
/* The same fit in stages: prepare (blocking + H2D, :279-337), run supersteps
   (the BulkIteration :341-344; continues the superstep counter across calls),
   and wait for completion.  Resume = mf_set_factors + mf_dsgd_set_superstep. */
int mf_dsgd_prepare(mf_ctx* ctx, const int32_t* users, const int32_t* items, const double* ratings,
                    int64_t n);
int mf_dsgd_run(mf_ctx* ctx, int64_t supersteps);
int mf_dsgd_superstep(mf_ctx* ctx, int64_t* done);
int mf_dsgd_set_superstep(mf_ctx* ctx, int64_t done);
/* Start the prepared fit over: factors back to their initial values (k x nextDouble of
   new Random(id ^ seed), DSGDforMF.scala:548-549) and the superstep counter to 0; blocking
   and the device schedule are kept.  mf_dsgd_run(iterations * numBlocks) then repeats fitSGD. */
int mf_dsgd_restart(mf_ctx* ctx);
int mf_sync(mf_ctx* ctx);

/* unblock (DSGDforMF.scala:245-255) -> factorsOption (MatrixFactorization.scala:64).
   Rows come back in ascending id order. In rank mode only the rows this rank owns. */
int mf_num_factors(mf_ctx* ctx, int side, int64_t* count);
int mf_get_factors(mf_ctx* ctx, int side, int32_t* ids_out, double* vecs_out, int64_t cap,
                   int64_t* written);
/* Overwrite (or, in online use, insert) factor rows (checkpoint restore). */
int mf_set_factors(mf_ctx* ctx, int side, const int32_t* ids, const double* vecs, int64_t n);
/* The context's parameters (e.g. the rank k a caller sizes factor buffers with). */
int mf_get_params(mf_ctx* ctx, mf_params* out);

/* Input and snapshots.
   mf_read_ratings: env.readCsvFile[(Int, Int, Double)](path) (DSGDforMF.scala:72) and MovieLens
   u.data: one "user<d>item<d>rating[<d>...]" record per line, d = delim (',' is Flink's default,
   '\t' u.data, 0 = any run of spaces / tabs / commas), the first skip_lines lines skipped, blank
   lines ignored, extra fields ignored.  users == NULL: only *n_out = record count.  A line
   that does not parse fails with MF_ERR_INVALID naming the line.
   mf_save_model / mf_load_model: the TemporaryPath persistence of the fit (DSGDforMF.scala:291-296,
   330-349) as one binary file: both factor sides (ids ascending, f64) and the superstep counter.
   Loading sets the factors (mf_set_factors semantics) and returns the stored counter; to resume
   a fit: mf_dsgd_prepare (same ratings), mf_load_model, mf_dsgd_set_superstep(counter),
   mf_dsgd_run. */
int mf_read_ratings(const char* path, char delim, int32_t skip_lines, int32_t* users, int32_t* items,
                    double* ratings, int64_t cap, int64_t* n_out);
int mf_save_model(mf_ctx* ctx, const char* path);
int mf_load_model(mf_ctx* ctx, const char* path, int64_t* superstep_out);

/* predictRating (MatrixFactorization.scala:239-274): inner-join semantics via found[]. */
int mf_predict(mf_ctx* ctx, const int32_t* users, const int32_t* items, int64_t n, double* out,
               uint8_t* found);
/* RMSE = sqrt(mean((r - p.q)^2)) over the inner-joined pairs (the reference has none). */
int mf_rmse(mf_ctx* ctx, const int32_t* users, const int32_t* items, const double* ratings,
            int64_t n, double* rmse, int64_t* matched);
/* empiricalRisk (MatrixFactorization.scala:133-192), duplicate-pair join semantics kept. */
int mf_empirical_risk(mf_ctx* ctx, const int32_t* users, const int32_t* items,
                      const double* ratings, int64_t n, double lambda, double* risk);

/* Exact updateLocalFactors replacement (DSGDforMF.scala:378-418) on caller buffers:
   users[nu x k], items[ni x k] are updated in place; omegas are per row.  Reentrant
   on disjoint buffers with distinct contexts, as Flink calls it per task slot. */
int mf_block_update(mf_ctx* ctx, const double* r, const int32_t* uidx, const int32_t* iidx,
                    int64_t len, double* users, const int32_t* uomega, int64_t nu, double* items,
                    const int32_t* iomega, int64_t ni, int k, int iteration, int rating_block_id,
                    int64_t seed, double lr, int lr_method, double lr_arg, double lambda);

/* Online micro-batch (FlinkOnlineMF.scala:112-137 via FactorUpdater.nextFactors;
   PSOfflineOnlineMF.scala:167-180 for MF_ONLINE_DELTA; OnlineSpark.scala:184-229 /
   OfflineSpark.scala:115-207 for MF_ONLINE_SPARK_SWEEP with num_partitions).
   Unseen ids are initialised with params.online_init.  Works on a fitted model too
   (combined offline + online).  Results equal sequential application in the
   flavour's order; touched counts are returned when the pointers are non-NULL. */
int mf_online_update(mf_ctx* ctx, const int32_t* users, const int32_t* items,
                     const double* ratings, int64_t n, int flavour, int num_partitions,
                     int64_t* touched_users, int64_t* touched_items);
/* mf_online_update plus the per-rating records the reference's operators emit, row j of the
   caller's n x k buffers (either may be NULL) for rating j in arrival order:
     MF_ONLINE_NEXT_FACTORS: user_out = nextUserVector, item_out = nextItemVector, the pair
       ItemOperator collects (fl/mf/online/FlinkOnlineMF.scala:131-135);
     MF_ONLINE_DELTA: user_out = userVec + deltaItemVec, the worker's ps.output
       (fl/mf/PSOfflineOnlineMF.scala:176, userVec before this rating's update), item_out =
       deltaItemVec, the vector pushed to the PS (:174).
   MF_ONLINE_SPARK_SWEEP emits only touched rows (OfflineSpark.scala:33-67): outputs must be NULL. */
int mf_online_update_out(mf_ctx* ctx, const int32_t* users, const int32_t* items,
                         const double* ratings, int64_t n, int flavour, int num_partitions,
                         int64_t* touched_users, int64_t* touched_items, double* user_out,
                         double* item_out);
/* Vectors for specific ids (found[j] = 0 for unknown ids). */
int mf_lookup(mf_ctx* ctx, int side, const int32_t* ids, int64_t n, double* vecs_out,
              uint8_t* found);

/* Statistics; profiling = 1 times every sweep-kernel launch with HIP events. */
int mf_set_profiling(mf_ctx* ctx, int on);
int mf_get_stats(mf_ctx* ctx, mf_stats* out);
int mf_reset_stats(mf_ctx* ctx);

/* JVM-compatible helpers used by the shim and tests (no GPU needed). */
int mf_jvm_shuffle(int64_t seed, int64_t len, int32_t* out);           /* scala.util.Random.shuffle */
int mf_jvm_block_of(int32_t id, int64_t seed, int32_t n_blocks, int32_t* out);  /* :531-533 */
int mf_jvm_random_factors(int64_t rng_seed, int32_t k, double* out);   /* k x nextDouble */
int mf_learning_rate(int method, double lr, int32_t iteration, double lambda, double arg,
                     double* out);

#ifdef __cplusplus
}
#endif
#endif /* MFHIP_H */
