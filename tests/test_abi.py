"""CPU-only checks of the drop-in boundary: libcvxg.so loads and exports exactly the C-ABI of include/cvxg.h."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cvxg.h")


def _header_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(cvxg_[a-z_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from cvx_amd import build as B
    B.build(force=False, verbose=False)
    from cvx_amd import _lib
    return _lib.load()


def test_header_declares_entry_points():
    syms = _header_symbols()
    for s in ["cvxg_create", "cvxg_destroy", "cvxg_set_objective", "cvxg_set_objective_kl", "cvxg_set_ineq", "cvxg_set_eq",
              "cvxg_newton_step", "cvxg_centering", "cvxg_barrier_solve", "cvxg_barrier_eval",
              "cvxg_newton_direction", "cvxg_last_error"]:
        assert s in syms


def test_library_exports_every_header_symbol(lib):
    from cvx_amd import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (cvxg_\w+)", out))
    missing = [s for s in _header_symbols() if s not in exported]
    assert not missing, missing
    assert set(_header_symbols()) == set(_lib.SIGNATURES), "ctypes table must mirror the header"


def test_version_and_no_gpu_behaviour(lib):
    import ctypes as C
    assert b"gfx950" in lib.cvxg_version()
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present: covered by the gpu tests")
    h = C.c_void_p()
    rc = lib.cvxg_create(0, 8, 8, 0, C.byref(h))
    assert rc != 0  # CVXG_E_HIP without a device, no crash, no CPU fallback
    msg = lib.cvxg_last_error(h)
    assert msg is not None
    if h.value:
        lib.cvxg_destroy(h)


def test_bad_arguments_rejected(lib):
    import ctypes as C
    from cvx_amd import _lib
    h = C.c_void_p()
    assert lib.cvxg_create(0, 0, 4, 0, C.byref(h)) == _lib.CVXG_E_DIM
    assert lib.cvxg_create(0, 4, 4, 4, C.byref(h)) == _lib.CVXG_E_DIM  # p < n (EqualityConstraint.scala:18-20)
    assert lib.cvxg_create(0, 1023 * 64 + 1, 4, 0, C.byref(h)) == _lib.CVXG_E_UNSUPPORTED
    assert lib.cvxg_newton_step(None, None, None) == _lib.CVXG_E_ARG
    assert lib.cvxg_set_option(None, _lib.OPTIONS["early_abort"], 0) == _lib.CVXG_E_ARG


def test_no_environment_switches_in_the_product():
    """The library reads no environment variable that changes arithmetic: the engine options go
    through cvxg_set_option; the only getenv calls left name the two tracing files."""
    import glob
    calls = []
    for f in glob.glob(os.path.join(ROOT, "cvx_amd", "csrc", "*")):
        calls += re.findall(r'getenv\("(\w+)"\)', open(f).read())
    assert set(calls) <= {"CVXG_DF_TRACE", "CVXG_RUIZ_TRACE"}, calls


# A stand-in for the few (nine) JNI declarations jni/cvxg_jni.c uses, with the JDK's C signatures (jni.h: JNIEnv is a
# pointer to the function table; jdoubleArray / jintArray are jarray = jobject).  A compile check of the glue only:
# it proves nothing about JVM linkage.
_JNI_STANDIN = r"""
#ifndef JNI_STANDIN_H
#define JNI_STANDIN_H
typedef int jint;
typedef long jlong;
typedef double jdouble;
typedef jint jsize;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jdoubleArray;
typedef jarray jintArray;
typedef jarray jlongArray;
struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv*, const char*);
  jint (*ThrowNew)(JNIEnv*, jclass, const char*);
  jstring (*NewStringUTF)(JNIEnv*, const char*);
  jsize (*GetArrayLength)(JNIEnv*, jarray);
  void (*GetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, jint*);
  void (*GetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, jlong*);
  void (*GetDoubleArrayRegion)(JNIEnv*, jdoubleArray, jsize, jsize, jdouble*);
  void (*SetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, const jint*);
  void (*SetDoubleArrayRegion)(JNIEnv*, jdoubleArray, jsize, jsize, const jdouble*);
};
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#endif
"""


def test_jni_glue_compiles_against_jni_declarations(tmp_path):
    (tmp_path / "jni.h").write_text(_JNI_STANDIN)
    src = os.path.join(ROOT, "jni", "cvxg_jni.c")
    r = subprocess.run(["gcc", "-std=c99", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-I", str(tmp_path), "-I",
                        os.path.join(ROOT, "include"), src], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_jni_glue_binds_every_scala_native_and_every_step_entry():
    """Every `@native def` of CvxgNative in INTEGRATION.md has its Java_cvx_gpu_CvxgNative_* function in the glue and
    vice versa; the per-t / per-step entry points a Scala-owned t-loop needs are among them."""
    c_src = open(os.path.join(ROOT, "jni", "cvxg_jni.c")).read()
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    c_names = set(re.findall(r"Java_cvx_gpu_CvxgNative_(\w+)\s*\(", c_src))
    scala_names = set(re.findall(r"@native def (\w+)", doc))
    assert c_names == scala_names, (c_names ^ scala_names)
    for s in ("centering", "centeringBegin", "centeringResume", "newtonStep", "newtonDirection", "barrierEval",
              "constraintValues", "activeSet", "setQuad", "batchBarrierSolve", "batchNewtonStep",
              "setObjectiveKLPrimal", "pdDirection"):
        assert s in c_names
    assert "GetPrimitiveArrayCritical" not in c_src  # no critical region spans a GPU call


# C-ABI entry points a Scala caller has no use for: instrumentation, the engine's A/B options and the host-only schedule
# dump
_JNI_EXEMPT = {"cvxg_set_timing", "cvxg_get_phase_times", "cvxg_get_phase_stats", "cvxg_get_counters", "cvxg_set_ruiz_lookahead",
               "cvxg_chol_schedule", "cvxg_set_option"}


def _camel(sym):
    """cvxg_set_objective_kl_primal -> setObjectiveKlPrimal (compared case-insensitively below)."""
    parts = sym[len("cvxg_"):].split("_")
    return parts[0] + "".join(p.capitalize() for p in parts[1:])


def test_jni_binds_every_reference_facing_entry_point():
    """Every cvxg_* the header declares has a Java_cvx_gpu_CvxgNative_* export in the glue and an @native def in
    INTEGRATION.md (names compared case-insensitively: setObjectiveKL for cvxg_set_objective_kl), except the listed
    diagnostics; and every export forwards to the entry point it is named after."""
    c_src = open(os.path.join(ROOT, "jni", "cvxg_jni.c")).read()
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    c_names = {n.lower(): n for n in re.findall(r"Java_cvx_gpu_CvxgNative_(\w+)\s*\(", c_src)}
    scala_names = {n.lower() for n in re.findall(r"@native def (\w+)", doc)}
    missing = []
    for sym in _header_symbols():
        if sym in _JNI_EXEMPT:
            continue
        key = _camel(sym).lower()
        if key not in c_names or key not in scala_names:
            missing.append(sym)
            continue
        body = c_src[c_src.index("Java_cvx_gpu_CvxgNative_" + c_names[key] + "("):]
        body = body[:body.index("\n}\n")]
        assert sym + "(" in body, f"{c_names[key]} does not call {sym}"
    assert not missing, missing
    assert not (_JNI_EXEMPT - set(_header_symbols())), "exempt names must exist in the header"


# Scala / Breeze names the glue uses that are not defined in the reference's own sources
_SCALA_LIB = {"Array", "ArrayBuffer", "AssertionError", "DenseMatrix", "DenseVector", "Divergence",
              "IllegalArgumentException", "Iterations", "MaxValue", "NotConvergedException", "RuntimeException", "Some",
              "_1", "collection", "cols", "data", "fill", "forall", "foreach", "getOrElse", "gpu", "isDefined",
              "isInstanceOf", "length", "linalg", "loadLibrary", "majorStride", "map", "mutable", "nonEmpty", "toArray",
              "toInt", "zipWithIndex"}
_SCALA_KW = {"if", "else", "for", "while", "match", "case", "new", "def", "val", "var", "return", "override", "yield",
             "until", "with", "extends"}
REF_SCALA = "/root/reference/src/main/scala/cvx"


@pytest.mark.skipif(not os.path.isdir(REF_SCALA), reason="reference sources not present (GPU box)")
def test_scala_glue_calls_only_defined_names():
    """Every name the Scala blocks of INTEGRATION.md call or select (f(..), x.f, new C) is defined in those blocks
    (def / val / object / class / parameter / pattern) or in the reference's own sources (src/main/scala/cvx), or is a
    Scala / Breeze library name.  Catches glue that calls helpers nobody defines (a maintainer pasting it would not
    compile).  Names only: scoping and types are not checked."""
    import glob
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    code = "\n".join(re.findall(r"```scala\n(.*?)```", doc, re.S))
    code = re.sub(r"/\*.*?\*/", "", code, flags=re.S)
    code = re.sub(r"//[^\n]*", "", code)
    code = re.sub(r'"[^"\n]*"', '""', code)
    defined = set(re.findall(r"\b(?:def|val|var|object|class|trait)\s+(\w+)", code))
    defined |= set(re.findall(r"[(,]\s*(\w+)\s*:", code))       # parameters
    defined |= set(re.findall(r"\b(\w+)\s*=>", code))           # lambda parameters
    for pat in re.findall(r"\(([^()]*(?:\([^()]*\)[^()]*)*)\)\s*<-", code):  # for-comprehension patterns
        defined |= set(re.findall(r"\w+", pat))
    defined |= set(re.findall(r"\b(\w+)\s*<-", code))
    ref = "".join(open(f).read() for f in glob.glob(os.path.join(REF_SCALA, "*.scala")))
    ref_defined = set(re.findall(r"\b(?:def|val|var|object|class|trait)\s+(\w+)", ref))
    ref_defined |= set(re.findall(r"[(,]\s*(\w+)\s*:", ref))    # constructor / case-class parameters
    used = set(re.findall(r"\b([A-Za-z_]\w*)\s*\(", code)) | set(re.findall(r"\.([A-Za-z_]\w*)", code))
    used |= set(re.findall(r"\bnew\s+(\w+)", code))
    unknown = sorted(u for u in used if u not in defined | ref_defined | _SCALA_LIB | _SCALA_KW)
    assert not unknown, unknown
    # the onDevice factory carries what its reduced override needs
    assert re.search(r"def onDevice\([^)]*device: Int\)", code, re.S)
