/*
 * mfhip_jni.c -- the JNI shim behind jni/MfHip.java.  Goes to
 * core/src/main/native/ in the reference tree; links libmfhip.so:
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I<repo>/include \
 *       mfhip_jni.c -L<repo>/large-scale-recommendation_amd/lib -lmfhip -Wl,-rpath,'$ORIGIN' \
 *       -o libmfhipjni.so
 * Every non-zero status becomes a java.lang.RuntimeException carrying mf_last_error(), which is
 * what the reference throws for the same conditions (MatrixFactorization.scala:189-190, 270-271).
 * Arrays are pinned with GetPrimitiveArrayCritical only around the copy-in / copy-out calls (the
 * library never retains host pointers).  tests/test_abi.py compiles this file against include/mfhip.h
 * (with a minimal jni.h stand-in, this image has no JDK) so every call matches the C ABI.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "mfhip.h"

static int check(JNIEnv* env, int st) {
  if (st != MF_OK) {
    jclass ex = (*env)->FindClass(env, "java/lang/RuntimeException");
    (*env)->ThrowNew(env, ex, mf_last_error());
  }
  return st;
}
#define PIN(a) ((a) ? (*env)->GetPrimitiveArrayCritical(env, (a), NULL) : NULL)
#define UNPIN(a, p, mode) \
  do {                    \
    if (a) (*env)->ReleasePrimitiveArrayCritical(env, (a), (p), (mode)); \
  } while (0)
#define JFN(name) Java_hu_sztaki_ilab_recom_core_gpu_MfHip_##name
#define CTX(h) ((mf_ctx*)(intptr_t)(h))

static void fill_params(mf_params* p, jint k, jint it, jdouble lambda, jdouble lr, jint lrm, jdouble lra, jint nb,
                        jlong seed, jboolean hs, jint mode) {
  mf_params_init(p);
  p->num_factors = k;
  p->iterations = it;
  p->lambda = lambda;
  p->learning_rate = lr;
  p->lr_method = lrm;
  p->lr_arg = lra;
  p->num_blocks = nb;
  p->seed = seed;
  p->has_seed = hs ? 1 : 0;
  p->mode = mode;
}

JNIEXPORT jlong JNICALL JFN(create)(JNIEnv* env, jclass c, jint k, jint it, jdouble lambda, jdouble lr, jint lrm,
                                    jdouble lra, jint nb, jlong seed, jboolean hs, jint mode, jdouble olr, jint oinit,
                                    jintArray devs) {
  mf_params p;
  fill_params(&p, k, it, lambda, lr, lrm, lra, nb, seed, hs, mode);
  p.online_learning_rate = olr;
  p.online_init = oinit;
  mf_ctx* ctx = NULL;
  jsize nd = devs ? (*env)->GetArrayLength(env, devs) : 0;
  jint* d = devs ? (*env)->GetIntArrayElements(env, devs, NULL) : NULL;
  int st = mf_create(&p, (const int*)d, nd ? nd : 1, &ctx);
  if (d) (*env)->ReleaseIntArrayElements(env, devs, d, JNI_ABORT);
  return check(env, st) == MF_OK ? (jlong)(intptr_t)ctx : 0;
}

JNIEXPORT jbyteArray JNICALL JFN(commUniqueId)(JNIEnv* env, jclass c) {
  uint8_t uid[MF_UID_BYTES];
  if (check(env, mf_comm_unique_id(uid)) != MF_OK) return NULL;
  jbyteArray out = (*env)->NewByteArray(env, MF_UID_BYTES);
  (*env)->SetByteArrayRegion(env, out, 0, MF_UID_BYTES, (const jbyte*)uid);
  return out;
}

JNIEXPORT jlong JNICALL JFN(createRank)(JNIEnv* env, jclass c, jint k, jint it, jdouble lambda, jdouble lr, jint lrm,
                                        jdouble lra, jint nb, jlong seed, jboolean hs, jint mode, jint dev,
                                        jint nranks, jint rank, jbyteArray uid) {
  mf_params p;
  fill_params(&p, k, it, lambda, lr, lrm, lra, nb, seed, hs, mode);
  uint8_t id[MF_UID_BYTES] = {0};
  (*env)->GetByteArrayRegion(env, uid, 0, MF_UID_BYTES, (jbyte*)id);
  mf_ctx* ctx = NULL;
  int st = mf_create_rank(&p, dev, nranks, rank, id, &ctx);
  return check(env, st) == MF_OK ? (jlong)(intptr_t)ctx : 0;
}

JNIEXPORT void JNICALL JFN(destroy)(JNIEnv* env, jclass c, jlong h) { check(env, mf_destroy(CTX(h))); }

typedef int (*ratings_fn)(mf_ctx*, const int32_t*, const int32_t*, const double*, int64_t);

static void with_ratings(JNIEnv* env, jlong h, jintArray u, jintArray i, jdoubleArray r, ratings_fn fn) {
  jsize n = (*env)->GetArrayLength(env, r);
  void *pu = PIN(u), *pi = PIN(i), *pr = PIN(r);
  int st = fn(CTX(h), (const int32_t*)pu, (const int32_t*)pi, (const double*)pr, n);
  UNPIN(r, pr, JNI_ABORT);
  UNPIN(i, pi, JNI_ABORT);
  UNPIN(u, pu, JNI_ABORT);
  check(env, st);
}

JNIEXPORT void JNICALL JFN(dsgdFit)(JNIEnv* env, jclass c, jlong h, jintArray u, jintArray i, jdoubleArray r) {
  with_ratings(env, h, u, i, r, mf_dsgd_fit);
}

JNIEXPORT void JNICALL JFN(dsgdPrepare)(JNIEnv* env, jclass c, jlong h, jintArray u, jintArray i, jdoubleArray r) {
  with_ratings(env, h, u, i, r, mf_dsgd_prepare);
}

JNIEXPORT void JNICALL JFN(dsgdRun)(JNIEnv* env, jclass c, jlong h, jlong supersteps) {
  check(env, mf_dsgd_run(CTX(h), supersteps));
}

JNIEXPORT void JNICALL JFN(dsgdRestart)(JNIEnv* env, jclass c, jlong h) { check(env, mf_dsgd_restart(CTX(h))); }

JNIEXPORT void JNICALL JFN(sync)(JNIEnv* env, jclass c, jlong h) { check(env, mf_sync(CTX(h))); }

JNIEXPORT jlong JNICALL JFN(numFactors)(JNIEnv* env, jclass c, jlong h, jint side) {
  int64_t n = 0;
  check(env, mf_num_factors(CTX(h), side, &n));
  return n;
}

JNIEXPORT jlong JNICALL JFN(getFactors)(JNIEnv* env, jclass c, jlong h, jint side, jintArray ids, jdoubleArray vecs) {
  int64_t w = 0;
  jsize cap = (*env)->GetArrayLength(env, ids);
  void *pi = PIN(ids), *pv = PIN(vecs);
  int st = mf_get_factors(CTX(h), side, (int32_t*)pi, (double*)pv, cap, &w);
  UNPIN(vecs, pv, 0);
  UNPIN(ids, pi, 0);
  check(env, st);
  return w;
}

JNIEXPORT void JNICALL JFN(setFactors)(JNIEnv* env, jclass c, jlong h, jint side, jintArray ids, jdoubleArray vecs) {
  jsize n = (*env)->GetArrayLength(env, ids);
  void *pi = PIN(ids), *pv = PIN(vecs);
  int st = mf_set_factors(CTX(h), side, (const int32_t*)pi, (const double*)pv, n);
  UNPIN(vecs, pv, JNI_ABORT);
  UNPIN(ids, pi, JNI_ABORT);
  check(env, st);
}

JNIEXPORT void JNICALL JFN(predict)(JNIEnv* env, jclass c, jlong h, jintArray u, jintArray i, jdoubleArray out,
                                    jbyteArray found) {
  jsize n = (*env)->GetArrayLength(env, u);
  void *pu = PIN(u), *pi = PIN(i), *po = PIN(out), *pf = PIN(found);
  int st = mf_predict(CTX(h), (const int32_t*)pu, (const int32_t*)pi, n, (double*)po, (uint8_t*)pf);
  UNPIN(found, pf, 0);
  UNPIN(out, po, 0);
  UNPIN(i, pi, JNI_ABORT);
  UNPIN(u, pu, JNI_ABORT);
  check(env, st);
}

JNIEXPORT jdouble JNICALL JFN(rmse)(JNIEnv* env, jclass c, jlong h, jintArray u, jintArray i, jdoubleArray r) {
  double rmse = 0;
  int64_t matched = 0;
  jsize n = (*env)->GetArrayLength(env, r);
  void *pu = PIN(u), *pi = PIN(i), *pr = PIN(r);
  int st = mf_rmse(CTX(h), (const int32_t*)pu, (const int32_t*)pi, (const double*)pr, n, &rmse, &matched);
  UNPIN(r, pr, JNI_ABORT);
  UNPIN(i, pi, JNI_ABORT);
  UNPIN(u, pu, JNI_ABORT);
  check(env, st);
  return rmse;
}

JNIEXPORT jdouble JNICALL JFN(empiricalRisk)(JNIEnv* env, jclass c, jlong h, jintArray u, jintArray i,
                                             jdoubleArray r, jdouble lambda) {
  double risk = 0;
  jsize n = (*env)->GetArrayLength(env, r);
  void *pu = PIN(u), *pi = PIN(i), *pr = PIN(r);
  int st = mf_empirical_risk(CTX(h), (const int32_t*)pu, (const int32_t*)pi, (const double*)pr, n, lambda, &risk);
  UNPIN(r, pr, JNI_ABORT);
  UNPIN(i, pi, JNI_ABORT);
  UNPIN(u, pu, JNI_ABORT);
  check(env, st);
  return risk;
}

JNIEXPORT void JNICALL JFN(blockUpdate)(JNIEnv* env, jclass c, jlong h, jdoubleArray r, jintArray uidx,
                                        jintArray iidx, jdoubleArray users, jintArray uom, jdoubleArray items,
                                        jintArray iom, jint k, jint iteration, jint rbid, jlong seed, jdouble lr,
                                        jint lrm, jdouble lra, jdouble lambda) {
  jsize len = (*env)->GetArrayLength(env, r);
  jsize nu = (*env)->GetArrayLength(env, uom), ni = (*env)->GetArrayLength(env, iom);
  void *pr = PIN(r), *pu = PIN(uidx), *pi = PIN(iidx), *pU = PIN(users), *pUo = PIN(uom), *pI = PIN(items),
       *pIo = PIN(iom);
  int st = mf_block_update(CTX(h), (const double*)pr, (const int32_t*)pu, (const int32_t*)pi, len, (double*)pU,
                           (const int32_t*)pUo, nu, (double*)pI, (const int32_t*)pIo, ni, k, iteration, rbid, seed, lr,
                           lrm, lra, lambda);
  UNPIN(iom, pIo, JNI_ABORT);
  UNPIN(items, pI, 0);
  UNPIN(uom, pUo, JNI_ABORT);
  UNPIN(users, pU, 0);
  UNPIN(iidx, pi, JNI_ABORT);
  UNPIN(uidx, pu, JNI_ABORT);
  UNPIN(r, pr, JNI_ABORT);
  check(env, st);
}

JNIEXPORT void JNICALL JFN(onlineUpdate)(JNIEnv* env, jclass c, jlong h, jintArray u, jintArray i, jdoubleArray r,
                                         jint flavour, jint parts) {
  jsize n = (*env)->GetArrayLength(env, r);
  void *pu = PIN(u), *pi = PIN(i), *pr = PIN(r);
  int st = mf_online_update(CTX(h), (const int32_t*)pu, (const int32_t*)pi, (const double*)pr, n, flavour, parts,
                            NULL, NULL);
  UNPIN(r, pr, JNI_ABORT);
  UNPIN(i, pi, JNI_ABORT);
  UNPIN(u, pu, JNI_ABORT);
  check(env, st);
}

JNIEXPORT void JNICALL JFN(onlineUpdateOut)(JNIEnv* env, jclass c, jlong h, jintArray u, jintArray i, jdoubleArray r,
                                            jint flavour, jdoubleArray uout, jdoubleArray iout) {
  jsize n = (*env)->GetArrayLength(env, r);
  void *pu = PIN(u), *pi = PIN(i), *pr = PIN(r), *puo = PIN(uout), *pio = PIN(iout);
  int st = mf_online_update_out(CTX(h), (const int32_t*)pu, (const int32_t*)pi, (const double*)pr, n, flavour, 0,
                                NULL, NULL, (double*)puo, (double*)pio);
  UNPIN(iout, pio, 0);
  UNPIN(uout, puo, 0);
  UNPIN(r, pr, JNI_ABORT);
  UNPIN(i, pi, JNI_ABORT);
  UNPIN(u, pu, JNI_ABORT);
  check(env, st);
}

JNIEXPORT void JNICALL JFN(lookup)(JNIEnv* env, jclass c, jlong h, jint side, jintArray ids, jdoubleArray out,
                                   jbyteArray found) {
  jsize n = (*env)->GetArrayLength(env, ids);
  void *pi = PIN(ids), *po = PIN(out), *pf = PIN(found);
  int st = mf_lookup(CTX(h), side, (const int32_t*)pi, n, (double*)po, (uint8_t*)pf);
  UNPIN(found, pf, 0);
  UNPIN(out, po, 0);
  UNPIN(ids, pi, JNI_ABORT);
  check(env, st);
}

JNIEXPORT jlong JNICALL JFN(countRatings)(JNIEnv* env, jclass c, jstring path, jchar d, jint skip) {
  const char* p = (*env)->GetStringUTFChars(env, path, NULL);
  int64_t n = 0;
  int st = mf_read_ratings(p, (char)d, skip, NULL, NULL, NULL, 0, &n);
  (*env)->ReleaseStringUTFChars(env, path, p);
  check(env, st);
  return n;
}

JNIEXPORT void JNICALL JFN(readRatings)(JNIEnv* env, jclass c, jstring path, jchar d, jint skip, jintArray u,
                                        jintArray i, jdoubleArray r) {
  const char* p = (*env)->GetStringUTFChars(env, path, NULL);
  jsize cap = (*env)->GetArrayLength(env, r);
  int64_t n = 0;
  void *pu = PIN(u), *pi = PIN(i), *pr = PIN(r);
  int st = mf_read_ratings(p, (char)d, skip, (int32_t*)pu, (int32_t*)pi, (double*)pr, cap, &n);
  UNPIN(r, pr, 0);
  UNPIN(i, pi, 0);
  UNPIN(u, pu, 0);
  (*env)->ReleaseStringUTFChars(env, path, p);
  check(env, st);
}

JNIEXPORT void JNICALL JFN(saveModel)(JNIEnv* env, jclass c, jlong h, jstring path) {
  const char* p = (*env)->GetStringUTFChars(env, path, NULL);
  int st = mf_save_model(CTX(h), p);
  (*env)->ReleaseStringUTFChars(env, path, p);
  check(env, st);
}

JNIEXPORT jlong JNICALL JFN(loadModel)(JNIEnv* env, jclass c, jlong h, jstring path) {
  const char* p = (*env)->GetStringUTFChars(env, path, NULL);
  int64_t step = 0;
  int st = mf_load_model(CTX(h), p, &step);
  (*env)->ReleaseStringUTFChars(env, path, p);
  check(env, st);
  return step;
}
