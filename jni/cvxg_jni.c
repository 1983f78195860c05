/*
 * cvxg_jni.c — JNI glue a maintainer of spyqqqdia/cvx adds to call the MI355X engine (include/cvxg.h)
 * from Scala.  Binds the native methods of `cvx.gpu.CvxgNative`.  Each method is a
 * thin forwarder: arrays are pinned with Get/ReleasePrimitiveArrayCritical only for the duration of
 * the call (the engine never retains host pointers), status codes are returned to Scala, where
 * `CvxgNative.check` maps them onto the reference's exceptions.
 *
 * Not built in this repository's CI: the image has no JDK (no jni.h).  Build recipe on a
 * host with a JDK:
 *   gcc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I../include \
 *       cvxg_jni.c -L../cvx_amd -lcvxg -Wl,-rpath,'$ORIGIN' -o libcvxg_jni.so
 */
#include <jni.h>
#include <stdint.h>

#include "cvxg.h"

#define CTX(h) ((cvxg_ctx*)(intptr_t)(h))

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
  return (*env)->NewStringUTF(env, cvxg_last_error(CTX(h)));
}

/* Breeze DenseMatrix data is column-major with majorStride = ld (row_major = 0); P may be null. */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_setObjective(JNIEnv* env, jclass cls, jlong h, jdoubleArray P,
                                                            jint ldP, jdoubleArray a, jdouble r) {
  (void)cls;
  double* pP = P ? (*env)->GetPrimitiveArrayCritical(env, P, 0) : 0;
  double* pa = (*env)->GetPrimitiveArrayCritical(env, a, 0);
  jint rc = cvxg_set_objective(CTX(h), pP, ldP, pa, r);
  (*env)->ReleasePrimitiveArrayCritical(env, a, pa, JNI_ABORT);
  if (pP) (*env)->ReleasePrimitiveArrayCritical(env, P, pP, JNI_ABORT);
  return rc;
}

/* Dist_KL dual objective (Duality.objF over Dist_KL): B = mat_B data (Breeze column-major, rowMajor = 0, ld =
 * majorStride), w = vec_w, R = vec_R(0). */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_setObjectiveKL(JNIEnv* env, jclass cls, jlong h, jdoubleArray B,
                                                              jint ldB, jint rowMajor, jint nout, jdoubleArray w,
                                                              jdouble R) {
  (void)cls;
  double* pB = (*env)->GetPrimitiveArrayCritical(env, B, 0);
  double* pw = (*env)->GetPrimitiveArrayCritical(env, w, 0);
  jint rc = cvxg_set_objective_kl(CTX(h), pB, ldB, rowMajor, nout, pw, R);
  (*env)->ReleasePrimitiveArrayCritical(env, w, pw, JNI_ABORT);
  (*env)->ReleasePrimitiveArrayCritical(env, B, pB, JNI_ABORT);
  return rc;
}

JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_setIneq(JNIEnv* env, jclass cls, jlong h, jdoubleArray A, jint ldA,
                                                       jint rowMajor, jdoubleArray r, jdoubleArray ub) {
  (void)cls;
  double* pA = (*env)->GetPrimitiveArrayCritical(env, A, 0);
  double* pr = (*env)->GetPrimitiveArrayCritical(env, r, 0);
  double* pu = (*env)->GetPrimitiveArrayCritical(env, ub, 0);
  jint rc = cvxg_set_ineq(CTX(h), pA, ldA, rowMajor, pr, pu);
  (*env)->ReleasePrimitiveArrayCritical(env, ub, pu, JNI_ABORT);
  (*env)->ReleasePrimitiveArrayCritical(env, r, pr, JNI_ABORT);
  (*env)->ReleasePrimitiveArrayCritical(env, A, pA, JNI_ABORT);
  return rc;
}

JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_setEq(JNIEnv* env, jclass cls, jlong h, jdoubleArray A, jint ld,
                                                     jint rowMajor, jdoubleArray b) {
  (void)cls;
  double* pA = (*env)->GetPrimitiveArrayCritical(env, A, 0);
  double* pb = (*env)->GetPrimitiveArrayCritical(env, b, 0);
  jint rc = cvxg_set_eq(CTX(h), pA, ld, rowMajor, pb);
  (*env)->ReleasePrimitiveArrayCritical(env, b, pb, JNI_ABORT);
  (*env)->ReleasePrimitiveArrayCritical(env, A, pA, JNI_ABORT);
  return rc;
}

JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_setX(JNIEnv* env, jclass cls, jlong h, jdoubleArray x) {
  (void)cls;
  double* px = (*env)->GetPrimitiveArrayCritical(env, x, 0);
  jint rc = cvxg_set_x(CTX(h), px);
  (*env)->ReleasePrimitiveArrayCritical(env, x, px, JNI_ABORT);
  return rc;
}

JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_getX(JNIEnv* env, jclass cls, jlong h, jdoubleArray x) {
  (void)cls;
  double* px = (*env)->GetPrimitiveArrayCritical(env, x, 0);
  jint rc = cvxg_get_x(CTX(h), px);
  (*env)->ReleasePrimitiveArrayCritical(env, x, px, 0);
  return rc;
}

/* barrierEval(h, t, x, f[1], g (nullable), H (nullable, n*n column-major)) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_barrierEval(JNIEnv* env, jclass cls, jlong h, jdouble t,
                                                           jdoubleArray x, jdoubleArray f, jdoubleArray g,
                                                           jdoubleArray H) {
  (void)cls;
  double fv = 0.0;
  double* px = (*env)->GetPrimitiveArrayCritical(env, x, 0);
  double* pg = g ? (*env)->GetPrimitiveArrayCritical(env, g, 0) : 0;
  double* pH = H ? (*env)->GetPrimitiveArrayCritical(env, H, 0) : 0;
  jint rc = cvxg_barrier_eval(CTX(h), t, px, &fv, pg, pH);
  if (pH) (*env)->ReleasePrimitiveArrayCritical(env, H, pH, 0);
  if (pg) (*env)->ReleasePrimitiveArrayCritical(env, g, pg, 0);
  (*env)->ReleasePrimitiveArrayCritical(env, x, px, JNI_ABORT);
  (*env)->SetDoubleArrayRegion(env, f, 0, 1, &fv);
  return rc;
}

/* barrierSolve(h, maxIter, params[6], termination, out[9]):
 * out = {dualityGap, equalityGap, newtonDecrement, normGrad, objective, iter, maxedOut, outerIters, steps} */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_barrierSolve(JNIEnv* env, jclass cls, jlong h, jint maxIter,
                                                            jdoubleArray jp, jint termination, jdoubleArray out) {
  (void)cls;
  cvxg_params p;
  cvxg_solution s;
  fill_params(env, jp, maxIter, &p);
  jint rc = cvxg_barrier_solve(CTX(h), &p, termination, &s);
  double o[9] = {s.duality_gap, s.equality_gap, s.newton_decrement, s.norm_grad, s.objective,
                 (double)s.iter, (double)s.maxed_out, (double)s.outer_iters, (double)s.newton_steps};
  (*env)->SetDoubleArrayRegion(env, out, 0, 9, o);
  return rc;
}

/* newtonDirection(h, maxIter, params[6], t, x, grad (nullable), dx, w (nullable)) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_newtonDirection(JNIEnv* env, jclass cls, jlong h, jint maxIter,
                                                               jdoubleArray jp, jdouble t, jdoubleArray x,
                                                               jdoubleArray grad, jdoubleArray dx, jdoubleArray w) {
  (void)cls;
  cvxg_params p;
  cvxg_step_info info;
  fill_params(env, jp, maxIter, &p);
  double* px = (*env)->GetPrimitiveArrayCritical(env, x, 0);
  double* pg = grad ? (*env)->GetPrimitiveArrayCritical(env, grad, 0) : 0;
  double* pd = (*env)->GetPrimitiveArrayCritical(env, dx, 0);
  double* pw = w ? (*env)->GetPrimitiveArrayCritical(env, w, 0) : 0;
  jint rc = cvxg_newton_direction(CTX(h), &p, t, px, pg, pd, pw, &info);
  if (pw) (*env)->ReleasePrimitiveArrayCritical(env, w, pw, 0);
  (*env)->ReleasePrimitiveArrayCritical(env, dx, pd, 0);
  if (pg) (*env)->ReleasePrimitiveArrayCritical(env, grad, pg, JNI_ABORT);
  (*env)->ReleasePrimitiveArrayCritical(env, x, px, JNI_ABORT);
  return rc;
}

/* pdSolve(h, maxIter, params[6], out[6]) -> PrimalDualSolver.solve on the device (cvxg_pd_solve) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_pdSolve(JNIEnv* env, jclass cls, jlong h, jint maxIter, jdoubleArray jp,
                                                       jdoubleArray out) {
  (void)cls;
  cvxg_params p;
  cvxg_pd_solution s;
  fill_params(env, jp, maxIter, &p);
  jint rc = cvxg_pd_solve(CTX(h), &p, &s);
  double o[6] = {s.duality_gap, s.norm_dual_residual, s.objective, (double)s.iter, (double)s.maxed_out,
                 (double)s.newton_steps};
  (*env)->SetDoubleArrayRegion(env, out, 0, 6, o);
  return rc;
}

/* getLambda(h, lambda[m]) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_getLambda(JNIEnv* env, jclass cls, jlong h, jdoubleArray lam) {
  (void)cls;
  double* pl = (*env)->GetPrimitiveArrayCritical(env, lam, 0);
  jint rc = cvxg_get_lambda(CTX(h), pl);
  (*env)->ReleasePrimitiveArrayCritical(env, lam, pl, 0);
  return rc;
}

/* setQuad(h, q, rows[q], P[q n n] row-major, ldP) -> QuadraticConstraint rows (cvxg_set_quad) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_setQuad(JNIEnv* env, jclass cls, jlong h, jint q, jintArray rows,
                                                       jdoubleArray P, jint ldP) {
  (void)cls;
  jint* pr = (*env)->GetPrimitiveArrayCritical(env, rows, 0);
  double* pp = (*env)->GetPrimitiveArrayCritical(env, P, 0);
  jint rc = cvxg_set_quad(CTX(h), q, (const int*)pr, pp, ldP);
  (*env)->ReleasePrimitiveArrayCritical(env, P, pp, JNI_ABORT);
  (*env)->ReleasePrimitiveArrayCritical(env, rows, pr, JNI_ABORT);
  return rc;
}

/* solutionSpace(dev, p, n, A[p n] column-major, b[p], z0[n], F[n (n-p)] column-major) -> SolutionSpace(A, b) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_solutionSpace(JNIEnv* env, jclass cls, jint dev, jint p, jint n,
                                                            jdoubleArray A, jdoubleArray b, jdoubleArray z0,
                                                            jdoubleArray F) {
  (void)cls;
  double* pA = (*env)->GetPrimitiveArrayCritical(env, A, 0);
  double* pb = (*env)->GetPrimitiveArrayCritical(env, b, 0);
  double* pz = (*env)->GetPrimitiveArrayCritical(env, z0, 0);
  double* pF = (*env)->GetPrimitiveArrayCritical(env, F, 0);
  jint rc = cvxg_solution_space(dev, p, n, pA, p, 0, pb, pz, pF, n);
  (*env)->ReleasePrimitiveArrayCritical(env, F, pF, 0);
  (*env)->ReleasePrimitiveArrayCritical(env, z0, pz, 0);
  (*env)->ReleasePrimitiveArrayCritical(env, b, pb, JNI_ABORT);
  (*env)->ReleasePrimitiveArrayCritical(env, A, pA, JNI_ABORT);
  return rc;
}

/* affineFrom(dst, src, z0[n], F[n k] column-major, ldF) -> BarrierSolver.affineTransformed (cvxg_affine_from) */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_affineFrom(JNIEnv* env, jclass cls, jlong dst, jlong src,
                                                         jdoubleArray z0, jdoubleArray F, jint ldF) {
  (void)cls;
  double* pz = (*env)->GetPrimitiveArrayCritical(env, z0, 0);
  double* pF = (*env)->GetPrimitiveArrayCritical(env, F, 0);
  jint rc = cvxg_affine_from(CTX(dst), CTX(src), pz, pF, ldF);
  (*env)->ReleasePrimitiveArrayCritical(env, F, pF, JNI_ABORT);
  (*env)->ReleasePrimitiveArrayCritical(env, z0, pz, JNI_ABORT);
  return rc;
}

/* affineParameter(h, x0[n], u0[k]) -> SolutionSpace.parameter;  affineMap(h, u[k] (nullable), x[n]) -> z0 + F u */
JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_affineParameter(JNIEnv* env, jclass cls, jlong h, jdoubleArray x0,
                                                              jdoubleArray u0) {
  (void)cls;
  double* px = (*env)->GetPrimitiveArrayCritical(env, x0, 0);
  double* pu = (*env)->GetPrimitiveArrayCritical(env, u0, 0);
  jint rc = cvxg_affine_parameter(CTX(h), px, pu);
  (*env)->ReleasePrimitiveArrayCritical(env, u0, pu, 0);
  (*env)->ReleasePrimitiveArrayCritical(env, x0, px, JNI_ABORT);
  return rc;
}

JNIEXPORT jint JNICALL Java_cvx_gpu_CvxgNative_affineMap(JNIEnv* env, jclass cls, jlong h, jdoubleArray u,
                                                        jdoubleArray x) {
  (void)cls;
  double* pu = u ? (*env)->GetPrimitiveArrayCritical(env, u, 0) : NULL;
  double* px = (*env)->GetPrimitiveArrayCritical(env, x, 0);
  jint rc = cvxg_affine_map(CTX(h), pu, px);
  (*env)->ReleasePrimitiveArrayCritical(env, x, px, 0);
  if (u) (*env)->ReleasePrimitiveArrayCritical(env, u, pu, JNI_ABORT);
  return rc;
}
