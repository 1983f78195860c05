/*
 * cvxg_jni.c — JNI glue a maintainer of spyqqqdia/cvx adds to call the MI355X engine (include/cvxg.h)
 * from Scala.  Binds the native methods of `cvx.gpu.CvxgNative`.  Each method is a
 * thin forwarder; status codes go back to Scala, where `CvxgNative.check` maps them onto the reference's
 * exceptions.
 *
 * Arrays are copied, never pinned: inputs with Get<Type>ArrayRegion into malloc'd buffers, outputs back with
 * Set<Type>ArrayRegion after the call.  The engine calls launch kernels and synchronize the stream (milliseconds
 * to seconds), which a JNI critical region must not span (it may stall the JVM's garbage collector).  The
 * copies cost one host memcpy of each array; the large ones (A, P) are passed once per problem.
 *
 * Not built in this repository's CI: the image has no JDK (no jni.h).  tests/test_abi.py
 * syntax-checks this file against a minimal stand-in for the few JNI types and functions it uses.  Build recipe
 * on a host with a JDK:
 *   gcc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I../include \
 *       cvxg_jni.c -L../cvx_amd -lcvxg -Wl,-rpath,'$ORIGIN' -o libcvxg_jni.so
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "cvxg.h"

#define CTX(h) ((cvxg_ctx*)(intptr_t)(h))

/* ---- array copies ------------------------------------------------------------------------------------- */

static void throw_oom(JNIEnv* env) {
  jclass c = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
  if (c) (*env)->ThrowNew(env, c, "cvxg_jni: host buffer allocation failed");
}

/* A malloc'd copy of a Java double[] (NULL for a null array).  *ok = 0 after an allocation failure (an
 * OutOfMemoryError is pending). */
static double* din(JNIEnv* env, jdoubleArray a, int* ok) {
  if (!a) return NULL;
  jsize n = (*env)->GetArrayLength(env, a);
  double* p = (double*)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
  if (!p) {
    throw_oom(env);
    *ok = 0;
    return NULL;
  }
  if (n > 0) (*env)->GetDoubleArrayRegion(env, a, 0, n, p);
  return p;
}

/* An uninitialised output buffer the size of a Java double[]. */
static double* dout(JNIEnv* env, jdoubleArray a, int* ok) {
  if (!a) return NULL;
  jsize n = (*env)->GetArrayLength(env, a);
  double* p = (double*)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
  if (!p) {
    throw_oom(env);
    *ok = 0;
  }
  return p;
}

/* Copy an output buffer back (on success) and free it. */
static void dput(JNIEnv* env, jdoubleArray a, double* p, jint rc) {
  if (!p) return;
  if (rc == CVXG_OK) (*env)->SetDoubleArrayRegion(env, a, 0, (*env)->GetArrayLength(env, a), p);
  free(p);
}

static void dfree(double* p) { free(p); }

static void fill_params(JNIEnv* env, jdoubleArray jp, jint maxIter, cvxg_params* p) {
  /* jp = {alpha, beta, tolSolver, tolEqSolve, tolFeas, delta}  (SolverParams.scala:24-32) */
  double v[6];
  (*env)->GetDoubleArrayRegion(env, jp, 0, 6, v);
  p->maxIter = maxIter;
  p->alpha = v[0];
  p->beta = v[1];
  p->tolSolver = v[2];
  p->tolEqSolve = v[3];
  p->tolFeas = v[4];
  p->delta = v[5];
}

/* cvxg_step_info as a double[23] (CvxgNative.StepInfo in INTEGRATION.md §2 reads it by these indices). */
#define STEP_INFO_LEN 23
static void step_info_row(const cvxg_step_info* s, double* o) {
  const double v[STEP_INFO_LEN] = {s->t, s->f, s->norm_grad, s->q, s->newton_decrement, s->hnorm, s->trust_radius,
                                   s->step, s->rel_err, s->min_diag, s->norm_grad_new, s->equality_gap,
                                   (double)s->backtracks_c, (double)s->backtracks_armijo, (double)s->fallback,
                                   (double)s->ruiz_sweeps, (double)s->regularized, (double)s->took_step,
                                   (double)s->done, (double)s->iter, (double)s->ls_fresh, (double)s->ls_ties,
                                   (double)s->small_pivot};
  for (int i = 0; i < STEP_INFO_LEN; ++i) o[i] = v[i];
}
static void put_step_info(JNIEnv* env, jdoubleArray out, const cvxg_step_info* s) {
  double o[STEP_INFO_LEN];
  step_info_row(s, o);
  if (out) (*env)->SetDoubleArrayRegion(env, out, 0, STEP_INFO_LEN, o);
}

/* ---- context -------------------------------------------------------------------------------------------- */

/* long create(int device, int n, int m, int p, int[] status) */
JNIEXPORT jlong JNICALL Java_cvx_gpu_CvxgNative_create(JNIEnv* env, jclass cls, jint dev, jint n, jint m, jint p,
                                                       jintArray jstatus) {
  (void)cls;
  cvxg_ctx* ctx = 0;
  jint rc = cvxg_create(dev, n, m, p, &ctx);
  (*env)->SetIntArrayRegion(env, jstatus, 0, 1, &rc);
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_cvx_gpu_CvxgNative_destroy(JNIEnv* env, jclass cls, jlong h) {
  (void)env;
  (void)cls;
  cvxg_destroy(CTX(h));
}

JNIEXPORT jstring JNICALL Java_cvx_gpu_CvxgNative_lastError(JNIEnv* env, jclass cls, jlong h) {
  (void)cls;
  const char* s = cvxg_last_error(CTX(h));
  return (*env)->NewStringUTF(env, s ? s : "");
}

JNIEXPORT jstring JNICALL Java_cvx_gpu_CvxgNative_version(JNIEnv* env, jclass cls) {
  (void)cls;
  const char* s = cvxg_version();
  return (*env)->NewStringUTF(env, s ? s : "");
}

/* ---- packing -------------------------------------------------------------------------------------------- */

/* Breeze DenseMatrix data is column-major with majorStride = ld (row_major = 0); P may be null. */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_setObjective(JNIEnv* env, jclass cls, jlong h, jdoubleArray P,
                                                            jint ldP, jdoubleArray a, jdouble r) {
  (void)cls;
  int ok = 1;
  double* pP = din(env, P, &ok);
  double* pa = din(env, a, &ok);
  jint rc = ok ? cvxg_set_objective(CTX(h), pP, ldP, pa, r) : CVXG_E_ARG;
  dfree(pa);
  dfree(pP);
  return rc;
}

/* Dist_KL dual objective (Duality.objF over Dist_KL): B = mat_B data (Breeze column-major, rowMajor = 0, ld =
 * majorStride), w = vec_w, R = vec_R(0). */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_setObjectiveKL(JNIEnv* env, jclass cls, jlong h, jdoubleArray B,
                                                              jint ldB, jint rowMajor, jint nout, jdoubleArray w,
                                                              jdouble R) {
  (void)cls;
  int ok = 1;
  double* pB = din(env, B, &ok);
  double* pw = din(env, w, &ok);
  jint rc = ok ? cvxg_set_objective_kl(CTX(h), pB, ldB, rowMajor, nout, pw, R) : CVXG_E_ARG;
  dfree(pw);
  dfree(pB);
  return rc;
}

/* Dist_KL.objectiveFunction(n) (Dist_KL.scala:223-239), the KL primal objective of kl_1 / kl_2: no data beyond the
 * outcome count n (cvxg_set_objective_kl_primal). */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_setObjectiveKLPrimal(JNIEnv* env, jclass cls, jlong h, jint nout) {
  (void)env;
  (void)cls;
  return cvxg_set_objective_kl_primal(CTX(h), nout);
}

JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_setIneq(JNIEnv* env, jclass cls, jlong h, jdoubleArray A, jint ldA,
                                                       jint rowMajor, jdoubleArray r, jdoubleArray ub) {
  (void)cls;
  int ok = 1;
  double* pA = din(env, A, &ok);
  double* pr = din(env, r, &ok);
  double* pu = din(env, ub, &ok);
  jint rc = ok ? cvxg_set_ineq(CTX(h), pA, ldA, rowMajor, pr, pu) : CVXG_E_ARG;
  dfree(pu);
  dfree(pr);
  dfree(pA);
  return rc;
}

/* setQuad(h, q, rows[q], P[q n n] row-major, ldP) -> QuadraticConstraint rows (cvxg_set_quad) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_setQuad(JNIEnv* env, jclass cls, jlong h, jint q, jintArray rows,
                                                       jdoubleArray P, jint ldP) {
  (void)cls;
  int ok = 1;
  jint* pr = (jint*)malloc((size_t)(q > 0 ? q : 1) * sizeof(jint));
  if (!pr) {
    throw_oom(env);
    return CVXG_E_ARG;
  }
  if (q > 0) (*env)->GetIntArrayRegion(env, rows, 0, q, pr);
  double* pp = din(env, P, &ok);
  jint rc = ok ? cvxg_set_quad(CTX(h), q, (const int*)pr, pp, ldP) : CVXG_E_ARG;
  dfree(pp);
  free(pr);
  return rc;
}

JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_setEq(JNIEnv* env, jclass cls, jlong h, jdoubleArray A, jint ld,
                                                     jint rowMajor, jdoubleArray b) {
  (void)cls;
  int ok = 1;
  double* pA = din(env, A, &ok);
  double* pb = din(env, b, &ok);
  jint rc = ok ? cvxg_set_eq(CTX(h), pA, ld, rowMajor, pb) : CVXG_E_ARG;
  dfree(pb);
  dfree(pA);
  return rc;
}

JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_setX(JNIEnv* env, jclass cls, jlong h, jdoubleArray x) {
  (void)cls;
  int ok = 1;
  double* px = din(env, x, &ok);
  jint rc = ok ? cvxg_set_x(CTX(h), px) : CVXG_E_ARG;
  dfree(px);
  return rc;
}

JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_getX(JNIEnv* env, jclass cls, jlong h, jdoubleArray x) {
  (void)cls;
  int ok = 1;
  double* px = dout(env, x, &ok);
  jint rc = ok ? cvxg_get_x(CTX(h), px) : CVXG_E_ARG;
  dput(env, x, px, rc);
  return rc;
}

/* ---- barrier oracles ------------------------------------------------------------------------------------ */

/* barrierEval(h, t, x, f[1], g (nullable), H (nullable, n*n column-major)) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_barrierEval(JNIEnv* env, jclass cls, jlong h, jdouble t,
                                                           jdoubleArray x, jdoubleArray f, jdoubleArray g,
                                                           jdoubleArray H) {
  (void)cls;
  int ok = 1;
  double fv = 0.0;
  double* px = din(env, x, &ok);
  double* pg = dout(env, g, &ok);
  double* pH = dout(env, H, &ok);
  jint rc = ok ? cvxg_barrier_eval(CTX(h), t, px, &fv, pg, pH) : CVXG_E_ARG;
  dput(env, H, pH, rc);
  dput(env, g, pg, rc);
  dfree(px);
  if (rc == CVXG_OK) (*env)->SetDoubleArrayRegion(env, f, 0, 1, &fv);
  return rc;
}

/* constraintValues(h, x, gx[m]) -> LinearConstraint.valueAt over the list */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_constraintValues(JNIEnv* env, jclass cls, jlong h, jdoubleArray x,
                                                                jdoubleArray gx) {
  (void)cls;
  int ok = 1;
  double* px = din(env, x, &ok);
  double* pg = dout(env, gx, &ok);
  jint rc = ok ? cvxg_constraint_values(CTX(h), px, pg) : CVXG_E_ARG;
  dput(env, gx, pg, rc);
  dfree(px);
  return rc;
}

/* activeSet(h, x, tol, idx[m], count[1]) -> Constraint.isActive over the list */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_activeSet(JNIEnv* env, jclass cls, jlong h, jdoubleArray x, jdouble tol,
                                                         jintArray idx, jintArray count) {
  (void)cls;
  int ok = 1;
  double* px = din(env, x, &ok);
  jsize cap = (*env)->GetArrayLength(env, idx);
  jint* pi = (jint*)malloc((size_t)(cap > 0 ? cap : 1) * sizeof(jint));
  if (!pi) {
    throw_oom(env);
    ok = 0;
  }
  jint cnt = 0;
  jint rc = ok ? cvxg_active_set(CTX(h), px, tol, (int*)pi, (int*)&cnt) : CVXG_E_ARG;
  if (rc == CVXG_OK) {
    if (cnt > 0) (*env)->SetIntArrayRegion(env, idx, 0, cnt, pi);
    (*env)->SetIntArrayRegion(env, count, 0, 1, &cnt);
  }
  free(pi);
  dfree(px);
  return rc;
}

/* ---- the hot path: one Newton direction, one inner iteration, one centering ------------------------------ */

/* newtonDirection(h, maxIter, params[6], t, x, grad (nullable), dx, w (nullable), info[23] (nullable)) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_newtonDirection(JNIEnv* env, jclass cls, jlong h, jint maxIter,
                                                               jdoubleArray jp, jdouble t, jdoubleArray x,
                                                               jdoubleArray grad, jdoubleArray dx, jdoubleArray w,
                                                               jdoubleArray info) {
  (void)cls;
  int ok = 1;
  cvxg_params p;
  cvxg_step_info si;
  fill_params(env, jp, maxIter, &p);
  double* px = din(env, x, &ok);
  double* pg = din(env, grad, &ok);
  double* pd = dout(env, dx, &ok);
  double* pw = dout(env, w, &ok);
  jint rc = ok ? cvxg_newton_direction(CTX(h), &p, t, px, pg, pd, pw, &si) : CVXG_E_ARG;
  dput(env, w, pw, rc);
  dput(env, dx, pd, rc);
  dfree(pg);
  dfree(px);
  if (rc == CVXG_OK) put_step_info(env, info, &si);
  return rc;
}

/* centeringBegin(h, t): a new UnconstrainedSolver / EqualityConstrainedSolver at t from the current iterate
 * (BarrierSolver.scala:97, 154) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_centeringBegin(JNIEnv* env, jclass cls, jlong h, jdouble t) {
  (void)env;
  (void)cls;
  return cvxg_centering_begin(CTX(h), t);
}

/* centeringResume(h, t, iter, trustRadius, grad (nullable)): the inner loop's state before iteration `iter` */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_centeringResume(JNIEnv* env, jclass cls, jlong h, jdouble t, jint iter,
                                                               jdouble radius, jdoubleArray grad) {
  (void)cls;
  int ok = 1;
  double* pg = din(env, grad, &ok);
  jint rc = ok ? cvxg_centering_resume(CTX(h), t, iter, radius, pg) : CVXG_E_ARG;
  dfree(pg);
  return rc;
}

/* newtonStep(h, maxIter, params[6], info[23]): one inner iteration on the device-resident iterate
 * (UnconstrainedSolver.scala:47-134 / EqualityConstrainedSolver.scala:60-111); info[18] = done */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_newtonStep(JNIEnv* env, jclass cls, jlong h, jint maxIter,
                                                          jdoubleArray jp, jdoubleArray info) {
  (void)cls;
  cvxg_params p;
  cvxg_step_info si;
  fill_params(env, jp, maxIter, &p);
  jint rc = cvxg_newton_step(CTX(h), &p, &si);
  if (rc == CVXG_OK) put_step_info(env, info, &si);
  return rc;
}

/* centering(h, maxIter, params[6], t, out[5]): the whole inner solve at t (UnconstrainedSolver.solve /
 * EqualityConstrainedSolver.solve); out = {iter, maxedOut, newtonDecrement, normGrad, equalityGap} */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_centering(JNIEnv* env, jclass cls, jlong h, jint maxIter,
                                                         jdoubleArray jp, jdouble t, jdoubleArray out) {
  (void)cls;
  cvxg_params p;
  cvxg_centering_info ci;
  fill_params(env, jp, maxIter, &p);
  jint rc = cvxg_centering(CTX(h), &p, t, &ci);
  if (rc == CVXG_OK) {
    double o[5] = {(double)ci.iter, (double)ci.maxed_out, ci.newton_decrement, ci.norm_grad, ci.equality_gap};
    (*env)->SetDoubleArrayRegion(env, out, 0, 5, o);
  }
  return rc;
}

/* barrierSolve(h, maxIter, params[6], termination, out[9]): the t-loop on the host of the engine (C / Python
 * callers; the Scala glue keeps its own t-loop and calls centering).
 * out = {dualityGap, equalityGap, newtonDecrement, normGrad, objective, iter, maxedOut, outerIters, steps} */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_barrierSolve(JNIEnv* env, jclass cls, jlong h, jint maxIter,
                                                            jdoubleArray jp, jint termination, jdoubleArray out) {
  (void)cls;
  cvxg_params p;
  cvxg_solution s;
  fill_params(env, jp, maxIter, &p);
  jint rc = cvxg_barrier_solve(CTX(h), &p, termination, &s);
  if (rc == CVXG_OK) {
    double o[9] = {s.duality_gap, s.equality_gap, s.newton_decrement, s.norm_grad, s.objective,
                   (double)s.iter, (double)s.maxed_out, (double)s.outer_iters, (double)s.newton_steps};
    (*env)->SetDoubleArrayRegion(env, out, 0, 9, o);
  }
  return rc;
}

/* batchBarrierSolve(handles[k], maxIter, params[6], termination, out[9 k], status[k]): config C5 from one JVM —
 * the barrier solves of k independent contexts (one per GPU) concurrently (cvxg_batch_barrier_solve) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_batchBarrierSolve(JNIEnv* env, jclass cls, jlongArray handles,
                                                                 jint maxIter, jdoubleArray jp, jint termination,
                                                                 jdoubleArray out, jintArray status) {
  (void)cls;
  cvxg_params p;
  fill_params(env, jp, maxIter, &p);
  jsize k = (*env)->GetArrayLength(env, handles);
  jlong* hv = (jlong*)malloc((size_t)(k > 0 ? k : 1) * sizeof(jlong));
  cvxg_ctx** cv = (cvxg_ctx**)malloc((size_t)(k > 0 ? k : 1) * sizeof(cvxg_ctx*));
  /* zeroed: an argument error (CVXG_E_ARG) returns before any instance writes its slot */
  cvxg_solution* sv = (cvxg_solution*)calloc((size_t)(k > 0 ? k : 1), sizeof(cvxg_solution));
  jint* st = (jint*)calloc((size_t)(k > 0 ? k : 1), sizeof(jint));
  double* o = (double*)malloc((size_t)(k > 0 ? 9 * k : 1) * sizeof(double));
  if (!hv || !cv || !sv || !st || !o) {
    free(hv), free(cv), free(sv), free(st), free(o);
    throw_oom(env);
    return CVXG_E_ARG;
  }
  if (k > 0) (*env)->GetLongArrayRegion(env, handles, 0, k, hv);
  for (jsize i = 0; i < k; ++i) cv[i] = CTX(hv[i]);
  jint rc = cvxg_batch_barrier_solve(k, cv, &p, termination, sv, (int*)st);
  for (jsize i = 0; i < k; ++i) {
    const cvxg_solution* s = &sv[i];
    double* r = o + 9 * i;
    r[0] = s->duality_gap, r[1] = s->equality_gap, r[2] = s->newton_decrement, r[3] = s->norm_grad;
    r[4] = s->objective, r[5] = (double)s->iter, r[6] = (double)s->maxed_out, r[7] = (double)s->outer_iters;
    r[8] = (double)s->newton_steps;
  }
  if (k > 0) {
    (*env)->SetDoubleArrayRegion(env, out, 0, 9 * k, o);
    (*env)->SetIntArrayRegion(env, status, 0, k, st);
  }
  free(hv), free(cv), free(sv), free(st), free(o);
  return rc;
}

/* batchNewtonStep(handles[k], maxIter, params[6], info[23 k], status[k]): one inner Newton iteration on each of k
 * independent contexts concurrently (cvxg_batch_newton_step); context i's cvxg_step_info at info[23 i ..] */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_batchNewtonStep(JNIEnv* env, jclass cls, jlongArray handles,
                                                               jint maxIter, jdoubleArray jp, jdoubleArray info,
                                                               jintArray status) {
  (void)cls;
  cvxg_params p;
  fill_params(env, jp, maxIter, &p);
  jsize k = (*env)->GetArrayLength(env, handles);
  jlong* hv = (jlong*)malloc((size_t)(k > 0 ? k : 1) * sizeof(jlong));
  cvxg_ctx** cv = (cvxg_ctx**)malloc((size_t)(k > 0 ? k : 1) * sizeof(cvxg_ctx*));
  /* zeroed: an argument error (CVXG_E_ARG) returns before any instance writes its slot */
  cvxg_step_info* sv = (cvxg_step_info*)calloc((size_t)(k > 0 ? k : 1), sizeof(cvxg_step_info));
  jint* st = (jint*)calloc((size_t)(k > 0 ? k : 1), sizeof(jint));
  double* o = (double*)malloc((size_t)(k > 0 ? STEP_INFO_LEN * k : 1) * sizeof(double));
  if (!hv || !cv || !sv || !st || !o) {
    free(hv), free(cv), free(sv), free(st), free(o);
    throw_oom(env);
    return CVXG_E_ARG;
  }
  if (k > 0) (*env)->GetLongArrayRegion(env, handles, 0, k, hv);
  for (jsize i = 0; i < k; ++i) cv[i] = CTX(hv[i]);
  jint rc = cvxg_batch_newton_step(k, cv, &p, sv, (int*)st);
  for (jsize i = 0; i < k; ++i) step_info_row(&sv[i], o + STEP_INFO_LEN * i);
  if (k > 0) {
    if (info) (*env)->SetDoubleArrayRegion(env, info, 0, STEP_INFO_LEN * k, o);
    (*env)->SetIntArrayRegion(env, status, 0, k, st);
  }
  free(hv), free(cv), free(sv), free(st), free(o);
  return rc;
}

/* ---- primal-dual solver --------------------------------------------------------------------------------- */

/* pdDirection(h, maxIter, params[6], t, x[n], lambda[m], dx[n] (nullable), dlambda[m] (nullable), info[9]
 * (nullable)): the PrimalDualSolver search direction (cvxg_pd_direction).  info = {t, s0, step, normResidual, relErr,
 * backtracks, fallback, ruizSweeps, regularized} */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_pdDirection(JNIEnv* env, jclass cls, jlong h, jint maxIter,
                                                           jdoubleArray jp, jdouble t, jdoubleArray x,
                                                           jdoubleArray lambda, jdoubleArray dx, jdoubleArray dlambda,
                                                           jdoubleArray info) {
  (void)cls;
  int ok = 1;
  cvxg_params p;
  cvxg_pd_step_info si;
  fill_params(env, jp, maxIter, &p);
  double* px = din(env, x, &ok);
  double* pl = din(env, lambda, &ok);
  double* pd = dout(env, dx, &ok);
  double* pdl = dout(env, dlambda, &ok);
  jint rc = ok ? cvxg_pd_direction(CTX(h), &p, t, px, pl, pd, pdl, &si) : CVXG_E_ARG;
  dput(env, dlambda, pdl, rc);
  dput(env, dx, pd, rc);
  dfree(pl);
  dfree(px);
  if (rc == CVXG_OK && info) {
    double o[9] = {si.t, si.s0, si.step, si.norm_residual, si.rel_err, (double)si.backtracks, (double)si.fallback,
                   (double)si.ruiz_sweeps, (double)si.regularized};
    (*env)->SetDoubleArrayRegion(env, info, 0, 9, o);
  }
  return rc;
}

/* pdDirectionEq(h, maxIter, params[6], t, x[n], lambda[m], nu[p], dx[n], dlambda[m], dnu[p] (outputs nullable),
 * info[9] (nullable)): the solve_withEQs search direction (cvxg_pd_direction_eq), info as pdDirection */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_pdDirectionEq(JNIEnv* env, jclass cls, jlong h, jint maxIter,
                                                             jdoubleArray jp, jdouble t, jdoubleArray x,
                                                             jdoubleArray lambda, jdoubleArray nu, jdoubleArray dx,
                                                             jdoubleArray dlambda, jdoubleArray dnu,
                                                             jdoubleArray info) {
  (void)cls;
  int ok = 1;
  cvxg_params p;
  cvxg_pd_step_info si;
  fill_params(env, jp, maxIter, &p);
  double* px = din(env, x, &ok);
  double* pl = din(env, lambda, &ok);
  double* pn = din(env, nu, &ok);
  double* pd = dout(env, dx, &ok);
  double* pdl = dout(env, dlambda, &ok);
  double* pdn = dout(env, dnu, &ok);
  jint rc = ok ? cvxg_pd_direction_eq(CTX(h), &p, t, px, pl, pn, pd, pdl, pdn, &si) : CVXG_E_ARG;
  dput(env, dnu, pdn, rc);
  dput(env, dlambda, pdl, rc);
  dput(env, dx, pd, rc);
  dfree(pn);
  dfree(pl);
  dfree(px);
  if (rc == CVXG_OK && info) {
    double o[9] = {si.t, si.s0, si.step, si.norm_residual, si.rel_err, (double)si.backtracks, (double)si.fallback,
                   (double)si.ruiz_sweeps, (double)si.regularized};
    (*env)->SetDoubleArrayRegion(env, info, 0, 9, o);
  }
  return rc;
}

/* pdSolve(h, maxIter, params[6], out[7]) -> PrimalDualSolver.solve on the device (cvxg_pd_solve; solve_withEQs when
 * the context has equality rows).  out = {gap, normResidual, objective, iter, maxedOut, newtonSteps, equalityGap},
 * also written on CVXG_E_LINESEARCH (the last accepted iterate; the Scala side throws LineSearchFailedException). */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_pdSolve(JNIEnv* env, jclass cls, jlong h, jint maxIter, jdoubleArray jp,
                                                       jdoubleArray out) {
  (void)cls;
  cvxg_params p;
  cvxg_pd_solution s;
  memset(&s, 0, sizeof(s));
  fill_params(env, jp, maxIter, &p);
  jint rc = cvxg_pd_solve(CTX(h), &p, &s);
  if (rc == CVXG_OK || rc == CVXG_E_LINESEARCH) {
    double o[7] = {s.duality_gap, s.norm_dual_residual, s.objective, (double)s.iter, (double)s.maxed_out,
                   (double)s.newton_steps, s.equality_gap};
    (*env)->SetDoubleArrayRegion(env, out, 0, 7, o);
  }
  return rc;
}

/* getNu(h, nu[p]) -> the equality multipliers after pdSolve (cvxg_get_nu) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_getNu(JNIEnv* env, jclass cls, jlong h, jdoubleArray nu) {
  (void)cls;
  int ok = 1;
  double* pn = dout(env, nu, &ok);
  jint rc = ok ? cvxg_get_nu(CTX(h), pn) : CVXG_E_ARG;
  dput(env, nu, pn, rc);
  return rc;
}

/* getLambda(h, lambda[m]) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_getLambda(JNIEnv* env, jclass cls, jlong h, jdoubleArray lam) {
  (void)cls;
  int ok = 1;
  double* pl = dout(env, lam, &ok);
  jint rc = ok ? cvxg_get_lambda(CTX(h), pl) : CVXG_E_ARG;
  dput(env, lam, pl, rc);
  return rc;
}

/* ---- affine re-parametrisation -------------------------------------------------------------------------- */

/* solutionSpace(dev, p, n, A[p n] column-major, b[p], z0[n], F[n (n-p)] column-major) -> SolutionSpace(A, b) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_solutionSpace(JNIEnv* env, jclass cls, jint dev, jint p, jint n,
                                                            jdoubleArray A, jdoubleArray b, jdoubleArray z0,
                                                            jdoubleArray F) {
  (void)cls;
  int ok = 1;
  double* pA = din(env, A, &ok);
  double* pb = din(env, b, &ok);
  double* pz = dout(env, z0, &ok);
  double* pF = dout(env, F, &ok);
  jint rc = ok ? cvxg_solution_space(dev, p, n, pA, p, 0, pb, pz, pF, n) : CVXG_E_ARG;
  dput(env, F, pF, rc);
  dput(env, z0, pz, rc);
  dfree(pb);
  dfree(pA);
  return rc;
}

/* affineFrom(dst, src, z0[n], F[n k] column-major, ldF) -> BarrierSolver.affineTransformed (cvxg_affine_from) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_affineFrom(JNIEnv* env, jclass cls, jlong dst, jlong src,
                                                         jdoubleArray z0, jdoubleArray F, jint ldF) {
  (void)cls;
  int ok = 1;
  double* pz = din(env, z0, &ok);
  double* pF = din(env, F, &ok);
  jint rc = ok ? cvxg_affine_from(CTX(dst), CTX(src), pz, pF, ldF) : CVXG_E_ARG;
  dfree(pF);
  dfree(pz);
  return rc;
}

/* affineParameter(h, x0[n], u0[k]) -> SolutionSpace.parameter;  affineMap(h, u[k] (nullable), x[n]) -> z0 + F u */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_affineParameter(JNIEnv* env, jclass cls, jlong h, jdoubleArray x0,
                                                              jdoubleArray u0) {
  (void)cls;
  int ok = 1;
  double* px = din(env, x0, &ok);
  double* pu = dout(env, u0, &ok);
  jint rc = ok ? cvxg_affine_parameter(CTX(h), px, pu) : CVXG_E_ARG;
  dput(env, u0, pu, rc);
  dfree(px);
  return rc;
}

JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_affineMap(JNIEnv* env, jclass cls, jlong h, jdoubleArray u,
                                                        jdoubleArray x) {
  (void)cls;
  int ok = 1;
  double* pu = din(env, u, &ok);
  double* px = dout(env, x, &ok);
  jint rc = ok ? cvxg_affine_map(CTX(h), pu, px) : CVXG_E_ARG;
  dput(env, x, px, rc);
  dfree(pu);
  return rc;
}
