// MfHip.java -- JNI entry points of libmfhip.so for the reference's Scala jobs (INTEGRATION.md).
// Goes to core/src/main/java/hu/sztaki/ilab/recom/core/gpu/MfHip.java in the reference tree; the
// native side is jni/mfhip_jni.c.  Every native method throws RuntimeException on a non-zero
// status, carrying mf_last_error() (MatrixFactorization.scala:189-190, 270-271 throw the same).
package hu.sztaki.ilab.recom.core.gpu;

public final class MfHip {
  static { System.loadLibrary("mfhipjni"); }   // links libmfhip.so

  public static final int MODE_DETERMINISTIC_F64 = 0, MODE_FAST_F32 = 1;
  // flink-ml LearningRateMethod (DSGDforMF.scala:10, 167-169)
  public static final int LR_DEFAULT = 0, LR_CONSTANT = 1, LR_BOTTOU = 2, LR_INVSCALING = 3, LR_XU = 4;
  public static final int SIDE_USER = 0, SIDE_ITEM = 1;
  public static final int ONLINE_NEXT_FACTORS = 0, ONLINE_DELTA = 1, ONLINE_SPARK_SWEEP = 2;
  public static final int INIT_PSEUDO_RANDOM = 0, INIT_SEEDED = 1;
  public static final int UID_BYTES = 128;

  // mf_create: params as MatrixFactorization.scala:201-223 / DSGDforMF.scala:163-169
  public static native long create(int k, int iterations, double lambda, double lr, int lrMethod,
                                   double lrArg, int numBlocks, long seed, boolean hasSeed, int mode,
                                   double onlineLr, int onlineInit, int[] deviceIds);
  // mf_comm_unique_id / mf_create_rank: one task per GPU, the id shipped by a broadcast variable
  public static native byte[] commUniqueId();
  public static native long createRank(int k, int iterations, double lambda, double lr, int lrMethod,
                                       double lrArg, int numBlocks, long seed, boolean hasSeed, int mode,
                                       int deviceId, int nranks, int rank, byte[] uid);
  public static native void destroy(long ctx);
  // fitSGD.fit (DSGDforMF.scala:262-357) in one call, or staged: prepare (blocking, :279-337),
  // run supersteps (the BulkIteration, :341-344), restart from the initial factors, sync
  public static native void dsgdFit(long ctx, int[] users, int[] items, double[] ratings);
  public static native void dsgdPrepare(long ctx, int[] users, int[] items, double[] ratings);
  public static native void dsgdRun(long ctx, long supersteps);
  public static native void dsgdRestart(long ctx);
  public static native void sync(long ctx);
  // unblock (DSGDforMF.scala:245-255) and checkpoint restore
  public static native long numFactors(long ctx, int side);
  public static native long getFactors(long ctx, int side, int[] idsOut, double[] vecsOut);
  public static native void setFactors(long ctx, int side, int[] ids, double[] vecs);
  // predictRating / RMSE / empiricalRisk (MatrixFactorization.scala:133-192, 239-274)
  public static native void predict(long ctx, int[] users, int[] items, double[] out, byte[] found);
  public static native double rmse(long ctx, int[] users, int[] items, double[] r);
  public static native double empiricalRisk(long ctx, int[] users, int[] items, double[] r, double lambda);
  // updateLocalFactors (DSGDforMF.scala:378-418) on the caller's flattened factor blocks
  public static native void blockUpdate(long ctx, double[] r, int[] uidx, int[] iidx,
                                        double[] users, int[] uomega, double[] items, int[] iomega,
                                        int k, int iteration, int ratingBlockId, long seed,
                                        double lr, int lrMethod, double lrArg, double lambda);
  // online micro-batches; onlineUpdateOut also returns every rating's emitted vectors
  // (FlinkOnlineMF.scala:131-135 / PSOfflineOnlineMF.scala:174-176), n x k each (may be null)
  public static native void onlineUpdate(long ctx, int[] users, int[] items, double[] r,
                                         int flavour, int numPartitions);
  public static native void onlineUpdateOut(long ctx, int[] users, int[] items, double[] r,
                                            int flavour, double[] userOut, double[] itemOut);
  public static native void lookup(long ctx, int side, int[] ids, double[] vecsOut, byte[] found);
  // env.readCsvFile[(Int, Int, Double)] replacement (DSGDforMF.scala:72)
  public static native long countRatings(String path, char delimiter, int skipLines);
  public static native void readRatings(String path, char delimiter, int skipLines, int[] users,
                                        int[] items, double[] ratings);
  // TemporaryPath persistence of the fit; loadModel returns the superstep counter
  public static native void saveModel(long ctx, String path);
  public static native long loadModel(long ctx, String path);
}
