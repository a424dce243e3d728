/*
 * sparkbam_jni.c -- the JNI shim a maintainer adds to spark-bam so its Scala host side
 * (modules bgzf / check / load / cli) calls libsparkbam_hip.so (include/sparkbam.h).
 *
 * Java class: org.hammerlab.bam.gpu.Native (jni/Native.scala).  Handles are jlongs; byte
 * buffers are direct ByteBuffers (no copies through the JVM heap).  Failures become the
 * reference's own exceptions, built with their real constructors (EXCEPTIONS below; the class
 * names and constructor descriptors are pinned against the reference's declarations by
 * tests/test_jni_names.py):
 *   SBH_E_HEADER_PARSE  -> org.hammerlab.bgzf.block.HeaderParseException(idx: Int, actual: Byte,
 *                          expected: Byte)   (bgzf/.../block/HeaderParseException.scala:6-11), from
 *                          sbh_last_error_detail's fields
 *   SBH_E_INFLATE_SIZE, SBH_E_BAD_ISIZE -> java.io.IOException(String) (bgzf/.../block/Stream.scala:52-54)
 *   SBH_E_INFLATE_DATA  -> java.util.zip.DataFormatException(String) (Inflater.inflate)
 *   SBH_E_TRUNCATED     -> java.io.EOFException(String)
 *   SBH_E_ARG           -> java.lang.IllegalArgumentException(String)
 *   SBH_E_NEED_HALO     -> org.hammerlab.bam.gpu.NeedHaloException(String) (the facade re-reads a
 *                          larger halo; never user-visible)
 *   SBH_E_NOT_FOUND, SBH_E_BAD_RECORD
 *                       -> org.hammerlab.bam.gpu.NativeException (below): the facades grow a shard
 *                          on them (a Pos or a record past the resident bytes)
 *   SBH_E_HEADER_SEARCH_FAILED, SBH_E_NO_READ_FOUND
 *                       -> org.hammerlab.bam.gpu.NativeException(status: Int, message: String,
 *                          fields: Array[Long]): their reference classes take the file's Path
 *                          (HeaderSearchFailedException(path, start, positionsAttempted),
 *                          bgzf/.../block/HeaderSearchFailedException.scala:7-12;
 *                          org.hammerlab.bam.spark.NoReadFoundException(path, start, maxReadSize),
 *                          check/.../spark/FindRecordStart.scala:66-71), which only the Scala
 *                          caller holds: Native.scala's `Native.rethrow(path)` builds them from the
 *                          fields {start, positionsAttempted} / {start, maxReadSize}
 *   anything else       -> java.lang.IllegalStateException(sbh_last_error)
 *
 * Built by jni/Makefile only when $JAVA_HOME/include/jni.h exists (no JDK in this image).
 */
#include <fcntl.h>
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "sparkbam.h"

#define CTX(x) ((sbh_ctx *)(intptr_t)(x))
#define SH(x) ((sbh_shard *)(intptr_t)(x))

#define STRING_CTOR "(Ljava/lang/String;)V"
#define NATIVE_EXCEPTION "org/hammerlab/bam/gpu/NativeException"
#define NATIVE_CTOR "(ILjava/lang/String;[J)V"

/* status -> the class thrown and the constructor it is built with */
static const struct {
  int rc;
  const char *cls, *ctor;
} EXCEPTIONS[] = {
    {SBH_E_HEADER_PARSE, "org/hammerlab/bgzf/block/HeaderParseException", "(IBB)V"},
    {SBH_E_HEADER_SEARCH_FAILED, NATIVE_EXCEPTION, NATIVE_CTOR},
    {SBH_E_NO_READ_FOUND, NATIVE_EXCEPTION, NATIVE_CTOR},
    {SBH_E_NOT_FOUND, NATIVE_EXCEPTION, NATIVE_CTOR},  /* a Pos past the shard: the facade grows it */
    {SBH_E_BAD_RECORD, NATIVE_EXCEPTION, NATIVE_CTOR}, /* a record past the shard (or malformed) */
    {SBH_E_INFLATE_SIZE, "java/io/IOException", STRING_CTOR},
    {SBH_E_BAD_ISIZE, "java/io/IOException", STRING_CTOR},
    {SBH_E_INFLATE_DATA, "java/util/zip/DataFormatException", STRING_CTOR},
    {SBH_E_TRUNCATED, "java/io/EOFException", STRING_CTOR},
    {SBH_E_ARG, "java/lang/IllegalArgumentException", STRING_CTOR},
    {SBH_E_NEED_HALO, "org/hammerlab/bam/gpu/NeedHaloException", STRING_CTOR},
};
static const char *const OTHER_EXCEPTION = "java/lang/IllegalStateException";

/* new cls(args...) thrown; a class or constructor that cannot be found leaves its
 * NoClassDefFoundError / NoSuchMethodError pending instead */
static void throw_new(JNIEnv *env, const char *cls, const char *ctor, int rc, const char *msg, const int64_t *f,
                      int nf) {
  jclass c = (*env)->FindClass(env, cls);
  if (!c) return;
  jmethodID init = (*env)->GetMethodID(env, c, "<init>", ctor);
  if (!init) return;
  jobject e = NULL;
  if (ctor[1] == 'I' && ctor[2] == 'B') { /* HeaderParseException(idx, actual, expected) */
    e = (*env)->NewObject(env, c, init, (jint)f[1], (jbyte)f[2], (jbyte)f[3]);
  } else if (ctor[1] == 'I') { /* NativeException(status, message, fields) */
    jstring m = (*env)->NewStringUTF(env, msg);
    jlongArray a = (*env)->NewLongArray(env, nf);
    if (!m || !a) return;
    (*env)->SetLongArrayRegion(env, a, 0, nf, (const jlong *)f);
    e = (*env)->NewObject(env, c, init, (jint)rc, m, a);
  } else {
    jstring m = (*env)->NewStringUTF(env, msg);
    if (!m) return;
    e = (*env)->NewObject(env, c, init, m);
  }
  if (e) (*env)->Throw(env, (jthrowable)e);
}

static void throw_status(JNIEnv *env, sbh_ctx *ctx, int rc) {
  const char *msg = ctx ? sbh_last_error(ctx) : "libsparkbam_hip";
  int64_t f[4] = {0, 0, 0, 0};
  int32_t code = 0;
  int nf = ctx ? (int)sbh_last_error_detail(ctx, &code, f, 4) : 0;
  if (code != rc || nf > 4) nf = code == rc ? 4 : 0; /* fields of another error are not this one's */
  const char *cls = OTHER_EXCEPTION, *ctor = STRING_CTOR;
  for (size_t i = 0; i < sizeof EXCEPTIONS / sizeof EXCEPTIONS[0]; ++i)
    if (EXCEPTIONS[i].rc == rc) cls = EXCEPTIONS[i].cls, ctor = EXCEPTIONS[i].ctor;
  if (rc == SBH_E_HEADER_PARSE && nf < 4) /* no byte to report: the status alone */
    cls = NATIVE_EXCEPTION, ctor = NATIVE_CTOR;
  throw_new(env, cls, ctor, rc, msg, f, nf);
}

/* status check: throws and returns 1 on failure */
static int failed(JNIEnv *env, jlong ctx, int rc) {
  if (rc == SBH_OK) return 0;
  throw_status(env, CTX(ctx), rc);
  return 1;
}

static void throw_arg(JNIEnv *env, const char *msg) {
  throw_new(env, "java/lang/IllegalArgumentException", STRING_CTOR, SBH_E_ARG, msg, NULL, 0);
}

/* The address of a direct ByteBuffer the library will read or write `need` bytes of.  A null
 * buffer gives NULL (an optional output is skipped, a required input is rejected by the
 * library).  A heap buffer (no address) or one shorter than `need` throws
 * IllegalArgumentException and sets *bad: the library never writes past the JVM's buffer. */
static void *direct_n(JNIEnv *env, jobject buf, uint64_t need, int *bad) {
  if (!buf) return NULL;
  void *p = (*env)->GetDirectBufferAddress(env, buf);
  const jlong cap = (*env)->GetDirectBufferCapacity(env, buf);
  if (!p || cap < 0) {
    throw_arg(env, "libsparkbam_hip needs a direct ByteBuffer");
    *bad = 1;
    return NULL;
  }
  if ((uint64_t)cap < need) {
    throw_arg(env, "ByteBuffer smaller than the bytes libsparkbam_hip reads or writes");
    *bad = 1;
    return NULL;
  }
  return p;
}

static int put_longs(JNIEnv *env, jlongArray out, const jlong *v, jsize n) {
  if ((*env)->GetArrayLength(env, out) < n) {
    throw_status(env, NULL, SBH_E_ARG);
    return 1;
  }
  (*env)->SetLongArrayRegion(env, out, 0, n, v);
  return 0;
}

/* ---- context / pinned memory ---- */
JNIEXPORT jlong JNICALL Java_org_hammerlab_bam_gpu_Native_00024_ctxCreate(JNIEnv *env, jobject self, jint dev) {
  sbh_ctx *ctx = NULL;
  int rc = sbh_ctx_create(dev, &ctx);
  if (rc) {
    throw_status(env, NULL, rc);
    return 0;
  }
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_ctxDestroy(JNIEnv *env, jobject self, jlong ctx) {
  sbh_ctx_destroy(CTX(ctx));
}

/* Page-locked host bytes as a direct ByteBuffer (compressed input for shardCreate/runStream). */
JNIEXPORT jobject JNICALL Java_org_hammerlab_bam_gpu_Native_00024_hostAlloc(JNIEnv *env, jobject self, jlong n) {
  void *p = NULL;
  int rc = sbh_host_alloc((uint64_t)n, &p);
  if (rc) {
    throw_status(env, NULL, rc);
    return NULL;
  }
  return (*env)->NewDirectByteBuffer(env, p, n);
}

JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_hostFree(JNIEnv *env, jobject self, jobject buf) {
  sbh_host_free(buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL);
}

/* ---- shards: compressed bytes [fileOffset, fileOffset + n) of a BGZF file ---- */
JNIEXPORT jlong JNICALL Java_org_hammerlab_bam_gpu_Native_00024_shardCreate(JNIEnv *env, jobject self, jlong ctx,
                                                                            jobject buf, jlong n, jlong fileOffset,
                                                                            jlong fileSize) {
  sbh_shard *sh = NULL;
  int bad = 0;
  const void *comp = direct_n(env, buf, (uint64_t)n, &bad);
  if (bad) return 0;
  if (failed(env, ctx, sbh_shard_create(CTX(ctx), comp, (uint64_t)n, (uint64_t)fileOffset, (uint64_t)fileSize, 0,
                                        &sh)))
    return 0;
  return (jlong)(intptr_t)sh;
}

JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_shardDestroy(JNIEnv *env, jobject self, jlong sh) {
  sbh_shard_destroy(SH(sh));
}

/* sbh_shard_load: the shard's resident bytes replaced by [fileOffset, fileOffset + n) of the same
 * file, its device buffers kept (a task thread's GpuSplitWorker reuses one shard for every split) */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_shardLoad(JNIEnv *env, jobject self, jlong ctx,
                                                                         jlong sh, jobject buf, jlong n,
                                                                         jlong fileOffset) {
  int bad = 0;
  const void *comp = direct_n(env, buf, (uint64_t)n, &bad);
  if (bad) return;
  (void)failed(env, ctx, sbh_shard_load(SH(sh), comp, (uint64_t)n, (uint64_t)fileOffset, 0));
}

/* FindBlockStart.apply (bgzf/.../block/FindBlockStart.scala:8-36) */
JNIEXPORT jlong JNICALL Java_org_hammerlab_bam_gpu_Native_00024_findBlockStart(JNIEnv *env, jobject self, jlong ctx,
                                                                               jlong sh, jlong start,
                                                                               jint blocksToCheck) {
  uint64_t out = 0;
  if (failed(env, ctx, sbh_find_block_start(SH(sh), (uint64_t)start, blocksToCheck, &out))) return -1;
  return (jlong)out;
}

/* MetadataStream + Stream inflate: out = {nBlocks, flatSize} */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_indexAndInflate(JNIEnv *env, jobject self, jlong ctx,
                                                                               jlong sh, jlong start,
                                                                               jlongArray out) {
  uint64_t nb = 0, fs = 0, bad = 0;
  if (failed(env, ctx, sbh_index(SH(sh), (uint64_t)start, &nb, &fs))) return;
  if (failed(env, ctx, sbh_inflate(SH(sh), &bad))) return;
  jlong v[2] = {(jlong)nb, (jlong)fs};
  put_longs(env, out, v, 2);
}

/* Block table as 6 longs per block: start, ustart, csize, hsize, usize, flags (Metadata.scala:6-8) */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_blocks(JNIEnv *env, jobject self, jlong ctx, jlong sh,
                                                                      jlong first, jlong count, jlongArray out) {
  sbh_block *b = (sbh_block *)malloc(sizeof(sbh_block) * (size_t)(count > 0 ? count : 1));
  if (!b) {
    throw_status(env, NULL, SBH_E_NOMEM);
    return;
  }
  if (!failed(env, ctx, sbh_get_blocks(SH(sh), (uint64_t)first, (uint64_t)count, b))) {
    jlong *v = (jlong *)malloc(sizeof(jlong) * 6 * (size_t)(count > 0 ? count : 1));
    if (v) {
      for (jlong i = 0; i < count; ++i) {
        v[6 * i] = (jlong)b[i].start, v[6 * i + 1] = (jlong)b[i].ustart, v[6 * i + 2] = b[i].csize;
        v[6 * i + 3] = b[i].hsize, v[6 * i + 4] = b[i].usize, v[6 * i + 5] = b[i].flags;
      }
      put_longs(env, out, v, (jsize)(6 * count));
      free(v);
    }
  }
  free(b);
}

/* Block.bytes on demand: flat [flat, flat + n) into a direct ByteBuffer */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_readFlat(JNIEnv *env, jobject self, jlong ctx,
                                                                        jlong sh, jlong flat, jlong n, jobject buf) {
  int bad = 0;
  uint8_t *out = (uint8_t *)direct_n(env, buf, (uint64_t)n, &bad);
  if (bad) return;
  failed(env, ctx, sbh_read_flat(SH(sh), (uint64_t)flat, (uint64_t)n, out));
}

JNIEXPORT jlong JNICALL Java_org_hammerlab_bam_gpu_Native_00024_flatOf(JNIEnv *env, jobject self, jlong ctx,
                                                                       jlong sh, jlong vpos) {
  uint64_t f = 0;
  if (failed(env, ctx, sbh_flat_of(SH(sh), (uint64_t)vpos >> 16, (uint32_t)(vpos & 0xffff), &f))) return -1;
  return (jlong)f;
}

JNIEXPORT jlong JNICALL Java_org_hammerlab_bam_gpu_Native_00024_posOf(JNIEnv *env, jobject self, jlong ctx, jlong sh,
                                                                      jlong flat) {
  uint64_t bp = 0;
  uint32_t off = 0;
  if (failed(env, ctx, sbh_pos_of(SH(sh), (uint64_t)flat, &bp, &off))) return -1;
  return (jlong)((bp << 16) | off);
}

/* flat image of Pos(fileOff, 0) as an exclusive bound: the first block at/after fileOff */
JNIEXPORT jlong JNICALL Java_org_hammerlab_bam_gpu_Native_00024_flatBound(JNIEnv *env, jobject self, jlong ctx,
                                                                          jlong sh, jlong fileOff) {
  uint64_t f = 0;
  if (failed(env, ctx, sbh_flat_bound(SH(sh), (uint64_t)fileOff, &f))) return -1;
  return (jlong)f;
}

/* ContigLengths (check/.../header/ContigLengths.scala) */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_setContigs(JNIEnv *env, jobject self, jlong ctx,
                                                                          jlong sh, jintArray lens) {
  const jsize n = (*env)->GetArrayLength(env, lens);
  jint *v = (*env)->GetIntArrayElements(env, lens, NULL);
  if (!v) return;
  const int rc = sbh_set_contigs(SH(sh), (const int32_t *)v, (int32_t)n);
  (*env)->ReleaseIntArrayElements(env, lens, v, JNI_ABORT);
  failed(env, ctx, rc);
}

/* eager.Checker over flat [begin, end): bit per position into `bits` (may be null) */
JNIEXPORT jlong JNICALL Java_org_hammerlab_bam_gpu_Native_00024_checkEager(JNIEnv *env, jobject self, jlong ctx,
                                                                           jlong sh, jlong begin, jlong end,
                                                                           jint readsToCheck, jobject bits) {
  uint64_t n_true = 0;
  int bad = 0;
  uint8_t *out = (uint8_t *)direct_n(env, bits, end > begin ? ((uint64_t)(end - begin) + 7) / 8 : 0, &bad);
  if (bad) return -1;
  if (failed(env, ctx, sbh_check_eager(SH(sh), (uint64_t)begin, (uint64_t)end, readsToCheck, out, &n_true)))
    return -1;
  return (jlong)n_true;
}

/* the eager bitmap the last checkEager / runShard left on the device, [begin, end) */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_eagerBits(JNIEnv *env, jobject self, jlong ctx,
                                                                         jlong sh, jlong begin, jlong end,
                                                                         jobject bits) {
  int bad = 0;
  uint8_t *out = (uint8_t *)direct_n(env, bits, end > begin ? ((uint64_t)(end - begin) + 7) / 8 : 0, &bad);
  if (bad) return;
  failed(env, ctx, sbh_eager_bits(SH(sh), (uint64_t)begin, (uint64_t)end, out));
}

/* full.Checker over flat [begin, end): words (may be null), counts 21*19, rbe 21*64, close
 * calls; out = {nSuccess, nClose} */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_checkFull(JNIEnv *env, jobject self, jlong ctx,
                                                                         jlong sh, jlong begin, jlong end,
                                                                         jint readsToCheck, jobject words,
                                                                         jobject counts, jobject rbe,
                                                                         jobject closeFlat, jobject closeWord,
                                                                         jlong closeCap, jlongArray out) {
  uint64_t ns = 0, nclose = 0;
  const uint64_t npos = end > begin ? (uint64_t)(end - begin) : 0, cc = closeCap > 0 ? (uint64_t)closeCap : 0;
  int bad = 0;
  uint32_t *w = (uint32_t *)direct_n(env, words, 4 * npos, &bad);
  uint64_t *c = bad ? NULL : (uint64_t *)direct_n(env, counts, 8ull * SBH_NNZ_MAX * 19, &bad);
  uint64_t *r = bad ? NULL : (uint64_t *)direct_n(env, rbe, 8ull * SBH_NNZ_MAX * SBH_RBE_MAX, &bad);
  uint64_t *cf = bad ? NULL : (uint64_t *)direct_n(env, closeFlat, 8 * cc, &bad);
  uint32_t *cw = bad ? NULL : (uint32_t *)direct_n(env, closeWord, 4 * cc, &bad);
  if (bad) return;
  if (failed(env, ctx, sbh_check_full(SH(sh), (uint64_t)begin, (uint64_t)end, readsToCheck, w, c, r, &ns, cf, cw,
                                      (cf || cw) ? cc : 0, &nclose)))
    return;
  jlong v[2] = {(jlong)ns, (jlong)nclose};
  put_longs(env, out, v, 2);
}

/* FindRecordStart.withDelta: out = {flat, delta} */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_findRecordStart(JNIEnv *env, jobject self, jlong ctx,
                                                                               jlong sh, jlong from,
                                                                               jint readsToCheck, jint maxReadSize,
                                                                               jlongArray out) {
  uint64_t f = 0;
  int32_t d = 0;
  if (failed(env, ctx, sbh_find_record_start(SH(sh), (uint64_t)from, readsToCheck, maxReadSize, &f, &d))) return;
  jlong v[2] = {(jlong)f, (jlong)d};
  put_longs(env, out, v, 2);
}

/* PosStream from a flat position: out = {records before endFlat, exit flat} */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_chainFrom(JNIEnv *env, jobject self, jlong ctx,
                                                                         jlong sh, jlong first, jlong endFlat,
                                                                         jlongArray out) {
  uint64_t n = 0, x = 0;
  if (failed(env, ctx, sbh_chain_from(SH(sh), (uint64_t)first, (uint64_t)endFlat, &n, &x))) return;
  jlong v[2] = {(jlong)n, (jlong)x};
  put_longs(env, out, v, 2);
}

/* loadSplitsAndReads for every split of a shard at once (CanLoadBam.scala:283-297,316-356):
 * starts/ends file offsets; out = 3 longs per split {status, firstVpos, count} */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_splitStarts(JNIEnv *env, jobject self, jlong ctx,
                                                                           jlong sh, jlongArray starts,
                                                                           jlongArray ends, jint blocksToCheck,
                                                                           jint readsToCheck, jint maxReadSize,
                                                                           jlongArray out) {
  const jsize n = (*env)->GetArrayLength(env, starts);
  if ((*env)->GetArrayLength(env, ends) != n) {
    throw_status(env, NULL, SBH_E_ARG);
    return;
  }
  uint64_t *buf = (uint64_t *)malloc(sizeof(uint64_t) * 4 * (size_t)(n > 0 ? n : 1));
  int32_t *status = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
  jlong *v = (jlong *)malloc(sizeof(jlong) * 3 * (size_t)(n > 0 ? n : 1));
  if (buf && status && v) {
    uint64_t *s = buf, *e = buf + n, *first = buf + 2 * n, *cnt = buf + 3 * n;
    (*env)->GetLongArrayRegion(env, starts, 0, n, (jlong *)s);
    (*env)->GetLongArrayRegion(env, ends, 0, n, (jlong *)e);
    if (!failed(env, ctx, sbh_split_starts(SH(sh), s, e, (uint64_t)n, blocksToCheck, readsToCheck, maxReadSize,
                                           first, cnt, status, NULL))) {
      for (jsize i = 0; i < n; ++i) v[3 * i] = status[i], v[3 * i + 1] = (jlong)first[i], v[3 * i + 2] = (jlong)cnt[i];
      put_longs(env, out, v, 3 * n);
    }
  } else {
    throw_status(env, NULL, SBH_E_NOMEM);
  }
  free(buf);
  free(status);
  free(v);
}

/* check-bam -s on the device: ranges as 2 longs each, truth records as vpos;
 * out = {tp, fp, fn, unknown}; fp/fn flat positions into direct buffers (may be null) */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_checkRecords(JNIEnv *env, jobject self, jlong ctx,
                                                                            jlong sh, jlongArray ranges,
                                                                            jint readsToCheck, jobject recVpos,
                                                                            jlong nRec, jobject fpFlat, jobject fnFlat,
                                                                            jlong cap, jlongArray out) {
  const jsize nr = (*env)->GetArrayLength(env, ranges) / 2;
  uint64_t *r = (uint64_t *)malloc(sizeof(uint64_t) * 2 * (size_t)(nr > 0 ? nr : 1));
  if (!r) {
    throw_status(env, NULL, SBH_E_NOMEM);
    return;
  }
  uint64_t *rb = r, *re = r + nr;
  for (jsize i = 0; i < nr; ++i) {
    jlong ab[2];
    (*env)->GetLongArrayRegion(env, ranges, 2 * i, 2, ab);
    rb[i] = (uint64_t)ab[0];
    re[i] = (uint64_t)ab[1];
  }
  uint64_t o[4] = {0, 0, 0, 0};
  const uint64_t cp = cap > 0 ? (uint64_t)cap : 0, nv = nRec > 0 ? (uint64_t)nRec : 0;
  int bad = 0;
  const uint64_t *rv = (const uint64_t *)direct_n(env, recVpos, 8 * nv, &bad);
  uint64_t *fp = bad ? NULL : (uint64_t *)direct_n(env, fpFlat, 8 * cp, &bad);
  uint64_t *fn = bad ? NULL : (uint64_t *)direct_n(env, fnFlat, 8 * cp, &bad);
  if (bad) {
    free(r);
    return;
  }
  if (!failed(env, ctx, sbh_check_records(SH(sh), rb, re, (uint64_t)nr, readsToCheck, rv, nv, o, fp, fp ? cp : 0, fn,
                                          fn ? cp : 0))) {
    jlong v[4] = {(jlong)o[0], (jlong)o[1], (jlong)o[2], (jlong)o[3]};
    put_longs(env, out, v, 4);
  }
  free(r);
}

/* The whole per-shard path (sbh_run_shard): out = {nBlocks, compBytes, flatBytes, nTrue,
 * firstVpos, count, exitFlat} */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_runShard(JNIEnv *env, jobject self, jlong ctx,
                                                                        jlong sh, jlong indexStart, jlong ownEnd,
                                                                        jint readsToCheck, jint maxReadSize,
                                                                        jlongArray out) {
  sbh_shard_result r;
  if (failed(env, ctx, sbh_run_shard(SH(sh), (uint64_t)indexStart, (uint64_t)ownEnd, readsToCheck, maxReadSize, &r)))
    return;
  jlong v[7] = {(jlong)r.n_blocks, (jlong)r.comp_bytes, (jlong)r.flat_bytes, (jlong)r.n_true,
                (jlong)r.first_vpos, (jlong)r.count, (jlong)r.exit_flat};
  put_longs(env, out, v, 7);
}

/* A split larger than HBM streamed through it (sbh_run_stream) from a (pinned) direct buffer:
 * out = {nWindows, compBytes, flatBytes, nTrue, count, firstVpos, exitVpos} */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_runStream(JNIEnv *env, jobject self, jlong ctx,
                                                                         jobject comp, jlong n, jlong fileOffset,
                                                                         jlong fileSize, jlong indexStart,
                                                                         jlong ownEnd, jlong window, jlong halo,
                                                                         jintArray contigs, jint readsToCheck,
                                                                         jint maxReadSize, jlongArray out) {
  int bad = 0;
  const void *src = direct_n(env, comp, (uint64_t)n, &bad);
  if (bad) return;
  const jsize nc = (*env)->GetArrayLength(env, contigs);
  jint *cl = (*env)->GetIntArrayElements(env, contigs, NULL);
  if (!cl) return;
  sbh_stream_result r;
  const int rc = sbh_run_stream(CTX(ctx), src, (uint64_t)n, (uint64_t)fileOffset, (uint64_t)fileSize,
                                (uint64_t)indexStart, (uint64_t)ownEnd, (uint64_t)window, (uint64_t)halo,
                                (const int32_t *)cl, (int32_t)nc, readsToCheck, maxReadSize, NULL, 0, &r);
  (*env)->ReleaseIntArrayElements(env, contigs, cl, JNI_ABORT);
  if (failed(env, ctx, rc)) return;
  jlong v[7] = {(jlong)r.n_windows, (jlong)r.comp_bytes, (jlong)r.flat_bytes, (jlong)r.n_true,
                (jlong)r.count, (jlong)r.first_vpos, (jlong)r.exit_vpos};
  put_longs(env, out, v, 7);
}

/* RecordStream + BAMRecordCodec.decode into columns: out = {n, nameBytes, cigarOps, bases,
 * auxBytes}; then recordsFetch fills one direct buffer per column (null = skip) */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_recordsScan(JNIEnv *env, jobject self, jlong ctx,
                                                                           jlong sh, jlong first, jlong endFlat,
                                                                           jlongArray out) {
  sbh_records_sizes z;
  if (failed(env, ctx, sbh_records_scan(SH(sh), (uint64_t)first, (uint64_t)endFlat, &z))) return;
  jlong v[5] = {(jlong)z.n, (jlong)z.name_bytes, (jlong)z.cigar_ops, (jlong)z.bases, (jlong)z.aux_bytes};
  put_longs(env, out, v, 5);
}

/* One FileSplit of loadReadsAndPositions in one call (sbh_split_records, CanLoadBam.scala:316-356):
 * out = {blockStart, nBlocks, flatSize, ownedFlat, firstFlat, firstVpos, nTrue, n, nameBytes,
 * cigarOps, bases, auxBytes}; out[7..11] are recordsFetch's sizes */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_splitRecords(JNIEnv *env, jobject self, jlong ctx,
                                                                            jlong sh, jlong start, jlong end,
                                                                            jint blocksToCheck, jint readsToCheck,
                                                                            jint maxReadSize, jboolean decode,
                                                                            jlongArray out) {
  sbh_split_records_result r;
  if (failed(env, ctx, sbh_split_records(SH(sh), (uint64_t)start, (uint64_t)end, blocksToCheck, readsToCheck,
                                         maxReadSize, decode ? 1 : 0, &r)))
    return;
  jlong v[12] = {(jlong)r.block_start, (jlong)r.n_blocks, (jlong)r.flat_size, (jlong)r.owned_flat,
                 (jlong)r.first_flat, (jlong)r.first_vpos, (jlong)r.n_true, (jlong)r.sizes.n,
                 (jlong)r.sizes.name_bytes, (jlong)r.sizes.cigar_ops, (jlong)r.sizes.bases, (jlong)r.sizes.aux_bytes};
  put_longs(env, out, v, 12);
}

JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_recordsFetch(JNIEnv *env, jobject self, jlong ctx,
                                                                            jlong sh, jlongArray sizes,
                                                                            jobjectArray cols) {
  /* 18 (or 19: + vpos) direct buffers in sbh_records_out field order, each checked against the
   * bytes of its column for the sizes recordsScan returned ({n, nameBytes, cigarOps, bases,
   * auxBytes}) */
  jlong z[5];
  if ((*env)->GetArrayLength(env, sizes) < 5) {
    throw_arg(env, "recordsFetch: sizes must hold recordsScan's 5 values");
    return;
  }
  (*env)->GetLongArrayRegion(env, sizes, 0, 5, z);
  const uint64_t n = (uint64_t)z[0], nm = (uint64_t)z[1], cg = (uint64_t)z[2], bs = (uint64_t)z[3], ax = (uint64_t)z[4];
  const uint64_t need[19] = {8 * n, 4 * n, 4 * n, 4 * n, 4 * n, 4 * n, 2 * n, 2 * n, n, 8 * (n + 1), 8 * (n + 1),
                             8 * (n + 1), 8 * (n + 1), nm, 4 * cg, bs, bs, ax, 8 * n};
  void *p[19] = {NULL};
  const jsize ncols = (*env)->GetArrayLength(env, cols) < 19 ? 18 : 19;
  int bad = 0;
  for (jsize i = 0; i < ncols && !bad; ++i)
    p[i] = direct_n(env, (*env)->GetObjectArrayElement(env, cols, i), need[i], &bad);
  if (bad) return;
  sbh_records_out o = {(uint64_t *)p[0], (int32_t *)p[1],  (int32_t *)p[2],  (int32_t *)p[3],  (int32_t *)p[4],
                       (int32_t *)p[5],  (uint16_t *)p[6], (uint16_t *)p[7], (uint8_t *)p[8],  (uint64_t *)p[9],
                       (uint64_t *)p[10], (uint64_t *)p[11], (uint64_t *)p[12], (char *)p[13], (uint32_t *)p[14],
                       (char *)p[15], (uint8_t *)p[16], (uint8_t *)p[17], (uint64_t *)p[18]};
  failed(env, ctx, sbh_records_fetch(SH(sh), &o));
}

/* sbh_run_stream2: a shard streamed through HBM with per-split results; splitOut = 3 longs per
 * split {status, firstVpos, count}; out = {nWindows, compBytes, flatBytes, nTrue, count,
 * firstVpos, exitVpos, crcBadBlocks} */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_runStreamSplits(
    JNIEnv *env, jobject self, jlong ctx, jobject comp, jlong n, jlong fileOffset, jlong fileSize, jlong indexStart,
    jlong ownEnd, jlong window, jlong halo, jintArray contigs, jint blocksToCheck, jint readsToCheck,
    jint maxReadSize, jboolean verifyCrc, jlongArray splitStarts, jlongArray splitEnds, jlongArray splitOut,
    jlongArray out) {
  int bad = 0;
  const void *src = direct_n(env, comp, (uint64_t)n, &bad);
  if (bad) return;
  const jsize ns = (*env)->GetArrayLength(env, splitStarts);
  if ((*env)->GetArrayLength(env, splitEnds) != ns || (*env)->GetArrayLength(env, splitOut) < 3 * ns) {
    throw_arg(env, "runStreamSplits: split arrays of different lengths");
    return;
  }
  uint64_t *buf = (uint64_t *)malloc(sizeof(uint64_t) * 4 * (size_t)(ns > 0 ? ns : 1));
  int32_t *status = (int32_t *)malloc(sizeof(int32_t) * (size_t)(ns > 0 ? ns : 1));
  jlong *v = (jlong *)malloc(sizeof(jlong) * 3 * (size_t)(ns > 0 ? ns : 1));
  const jsize nc = (*env)->GetArrayLength(env, contigs);
  jint *cl = (*env)->GetIntArrayElements(env, contigs, NULL);
  if (!buf || !status || !v || !cl) {
    if (cl) (*env)->ReleaseIntArrayElements(env, contigs, cl, JNI_ABORT);
    free(buf), free(status), free(v);
    if (!cl) return;
    throw_status(env, NULL, SBH_E_NOMEM);
    return;
  }
  uint64_t *st = buf, *en = buf + ns, *first = buf + 2 * ns, *cnt = buf + 3 * ns;
  (*env)->GetLongArrayRegion(env, splitStarts, 0, ns, (jlong *)st);
  (*env)->GetLongArrayRegion(env, splitEnds, 0, ns, (jlong *)en);
  sbh_stream_opts o = {0};
  o.window = (uint64_t)window;
  o.halo = (uint64_t)halo;
  o.reads_to_check = readsToCheck;
  o.max_read_size = maxReadSize;
  o.bgzf_blocks_to_check = blocksToCheck;
  o.verify_crc = verifyCrc ? 1 : 0;
  o.split_start = st, o.split_end = en, o.n_splits = (uint64_t)ns;
  o.split_first_vpos = first, o.split_count = cnt, o.split_status = status;
  sbh_stream_result r;
  const int rc = sbh_run_stream2(CTX(ctx), src, (uint64_t)n, (uint64_t)fileOffset, (uint64_t)fileSize,
                                 (uint64_t)indexStart, (uint64_t)ownEnd, (const int32_t *)cl, (int32_t)nc, &o, &r);
  (*env)->ReleaseIntArrayElements(env, contigs, cl, JNI_ABORT);
  if (!failed(env, ctx, rc)) {
    for (jsize i = 0; i < ns; ++i) v[3 * i] = status[i], v[3 * i + 1] = (jlong)first[i], v[3 * i + 2] = (jlong)cnt[i];
    if (!put_longs(env, splitOut, v, 3 * ns)) {
      jlong w[8] = {(jlong)r.n_windows, (jlong)r.comp_bytes, (jlong)r.flat_bytes, (jlong)r.n_true,
                    (jlong)r.count, (jlong)r.first_vpos, (jlong)r.exit_vpos, (jlong)r.crc_bad_blocks};
      put_longs(env, out, w, 8);
    }
  }
  free(buf), free(status), free(v);
}

/* The BGZF writer (sbh_bgzf_compress_level; level 5 = htsjdk's exact bytes) */
JNIEXPORT jlong JNICALL Java_org_hammerlab_bam_gpu_Native_00024_bgzfBound(JNIEnv *env, jobject self, jlong n) {
  return (jlong)sbh_bgzf_compress_bound((uint64_t)n);
}

JNIEXPORT jlong JNICALL Java_org_hammerlab_bam_gpu_Native_00024_bgzfCompress(JNIEnv *env, jobject self, jlong ctx,
                                                                             jobject src, jlong n, jint level,
                                                                             jobject out) {
  const uint64_t cap = sbh_bgzf_compress_bound((uint64_t)n);
  int bad = 0;
  const void *in = direct_n(env, src, (uint64_t)n, &bad);
  uint8_t *o = bad ? NULL : (uint8_t *)direct_n(env, out, cap, &bad);
  if (bad) return -1;
  uint64_t size = 0, nb = 0;
  if (failed(env, ctx, sbh_bgzf_compress_level(CTX(ctx), in, (uint64_t)n, 0, level, o, cap, &size, &nb, NULL)))
    return -1;
  return (jlong)size;
}

/* ---- files larger than a ByteBuffer: the file mapped read-only by the shim ---- */
typedef struct {
  void *p;
  uint64_t n;
} Mapped;

/* path -> read-only mapping of the whole (local) file; throws IOException on failure */
static int map_file(JNIEnv *env, jstring path, Mapped *m) {
  m->p = NULL, m->n = 0;
  const char *s = (*env)->GetStringUTFChars(env, path, NULL);
  if (!s) return 1;
  int fd = open(s, O_RDONLY);
  struct stat st;
  char msg[512];
  int ok = fd >= 0 && fstat(fd, &st) == 0;
  if (ok && st.st_size > 0) {
    m->n = (uint64_t)st.st_size;
    m->p = mmap(NULL, m->n, PROT_READ, MAP_PRIVATE, fd, 0);
    ok = m->p != MAP_FAILED;
    if (!ok) m->p = NULL;
  }
  snprintf(msg, sizeof msg, "%s: cannot map the file", s);
  if (fd >= 0) close(fd);
  (*env)->ReleaseStringUTFChars(env, path, s);
  if (!ok) throw_new(env, "java/io/IOException", STRING_CTOR, 0, msg, NULL, 0);
  return !ok;
}

static void unmap_file(Mapped *m) {
  if (m->p) munmap(m->p, m->n);
}

/* Blocks.apply's unindexed branch (check/.../check/Blocks.scala:141-206): FindBlockStart per
 * split, then MetadataStream to the split's end, windows through HBM (sbh_find_blocks).
 * Returns 4 longs per block {split index, start, compressedSize, uncompressedSize}. */
JNIEXPORT jlongArray JNICALL Java_org_hammerlab_bam_gpu_Native_00024_findBlocks(JNIEnv *env, jobject self, jlong ctx,
                                                                                jstring path, jlongArray starts,
                                                                                jlongArray ends, jint blocksToCheck,
                                                                                jlong window) {
  const jsize ns = (*env)->GetArrayLength(env, starts);
  if ((*env)->GetArrayLength(env, ends) != ns) {
    throw_arg(env, "findBlocks: split starts and ends of different lengths");
    return NULL;
  }
  Mapped m;
  if (map_file(env, path, &m)) return NULL;
  uint64_t *se = (uint64_t *)malloc(sizeof(uint64_t) * 2 * (size_t)(ns > 0 ? ns : 1));
  uint64_t cap = m.n / 16384 + 4096, n = 0; /* BAM blocks average 15-25 KB; regrown if short */
  sbh_block *out = NULL;
  jlongArray res = NULL;
  if (!se) {
    throw_status(env, NULL, SBH_E_NOMEM);
    goto done;
  }
  (*env)->GetLongArrayRegion(env, starts, 0, ns, (jlong *)se);
  (*env)->GetLongArrayRegion(env, ends, 0, ns, (jlong *)(se + ns));
  for (;;) {
    free(out);
    out = (sbh_block *)malloc(sizeof(sbh_block) * (size_t)cap);
    if (!out) {
      throw_status(env, NULL, SBH_E_NOMEM);
      goto done;
    }
    if (failed(env, ctx, sbh_find_blocks(CTX(ctx), m.p, m.n, se, se + ns, (uint64_t)ns, blocksToCheck,
                                         (uint64_t)window, out, cap, &n)))
      goto done;
    if (n <= cap) break;
    cap = n;
  }
  res = (*env)->NewLongArray(env, (jsize)(4 * n));
  if (res) {
    jlong *v = (jlong *)malloc(sizeof(jlong) * 4 * (size_t)(n ? n : 1));
    if (!v) {
      throw_status(env, NULL, SBH_E_NOMEM);
      res = NULL;
      goto done;
    }
    for (uint64_t i = 0; i < n; ++i) /* (sbh_find_blocks: ustart holds the split index) */
      v[4 * i] = (jlong)out[i].ustart, v[4 * i + 1] = (jlong)out[i].start, v[4 * i + 2] = out[i].csize,
      v[4 * i + 3] = out[i].usize;
    (*env)->SetLongArrayRegion(env, res, 0, (jsize)(4 * n), v);
    free(v);
  }
done:
  free(out);
  free(se);
  unmap_file(&m);
  return res;
}

/* check-bam -s / full-check over Blocks.apply's blocks of a file of any size
 * (cli/.../CallPartition.scala:23-54, cli/.../full/FullCheck.scala:65-86; sbh_check_stream):
 * blocks = file offsets of the block starts, ascending; truthVpos (direct, n_truth longs, or
 * null) = the `.records` positions; fp/fn vpos and the full aggregation into direct buffers
 * (null = skipped).  out = {nWindows, positions, compBytes, nTrue, tp, fp, fn, unknown,
 * nSuccess, nClose, haloFinal}. */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_checkStream(
    JNIEnv *env, jobject self, jlong ctx, jstring path, jintArray contigs, jlongArray blocks, jobject truthVpos,
    jlong nTruth, jboolean full, jlong window, jlong halo, jint readsToCheck, jobject fpVpos, jobject fnVpos,
    jlong mismatchCap, jobject counts, jobject rbe, jobject closeVpos, jobject closeWord, jlong closeCap,
    jlongArray out) {
  const jsize nb = (*env)->GetArrayLength(env, blocks);
  const uint64_t nt = nTruth > 0 ? (uint64_t)nTruth : 0, mc = mismatchCap > 0 ? (uint64_t)mismatchCap : 0,
                 cc = closeCap > 0 ? (uint64_t)closeCap : 0;
  int bad = 0;
  sbh_check_opts o = {0};
  o.window = (uint64_t)window, o.halo = (uint64_t)halo, o.reads_to_check = readsToCheck, o.full = full ? 1 : 0;
  o.truth_vpos = (const uint64_t *)direct_n(env, truthVpos, 8 * nt, &bad);
  o.n_truth = o.truth_vpos ? nt : 0;
  o.fp_vpos = bad ? NULL : (uint64_t *)direct_n(env, fpVpos, 8 * mc, &bad);
  o.fn_vpos = bad ? NULL : (uint64_t *)direct_n(env, fnVpos, 8 * mc, &bad);
  o.fp_cap = o.fp_vpos ? mc : 0, o.fn_cap = o.fn_vpos ? mc : 0;
  o.counts = bad ? NULL : (uint64_t *)direct_n(env, counts, 8ull * SBH_NNZ_MAX * 19, &bad);
  o.rbe_hist = bad ? NULL : (uint64_t *)direct_n(env, rbe, 8ull * SBH_NNZ_MAX * SBH_RBE_MAX, &bad);
  o.close_vpos = bad ? NULL : (uint64_t *)direct_n(env, closeVpos, 8 * cc, &bad);
  o.close_word = bad ? NULL : (uint32_t *)direct_n(env, closeWord, 4 * cc, &bad);
  o.close_cap = (o.close_vpos && o.close_word) ? cc : 0;
  if (bad) return;
  if (o.full && (!o.counts || !o.rbe_hist)) {
    throw_arg(env, "checkStream: full needs the counts and rbe buffers");
    return;
  }
  uint64_t *bl = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(nb > 0 ? nb : 1));
  if (!bl) {
    throw_status(env, NULL, SBH_E_NOMEM);
    return;
  }
  (*env)->GetLongArrayRegion(env, blocks, 0, nb, (jlong *)bl);
  o.blocks = bl, o.n_blocks = (uint64_t)nb;
  const jsize nc = (*env)->GetArrayLength(env, contigs);
  jint *cl = (*env)->GetIntArrayElements(env, contigs, NULL);
  Mapped m = {NULL, 0};
  if (cl && !map_file(env, path, &m)) {
    sbh_check_result r;
    const int rc = sbh_check_stream(CTX(ctx), m.p, m.n, (const int32_t *)cl, (int32_t)nc, &o, &r);
    if (!failed(env, ctx, rc)) {
      jlong v[11] = {(jlong)r.n_windows, (jlong)r.positions, (jlong)r.comp_bytes, (jlong)r.n_true, (jlong)r.tp,
                     (jlong)r.fp, (jlong)r.fn, (jlong)r.unknown, (jlong)r.n_success, (jlong)r.n_close,
                     (jlong)r.halo_final};
      put_longs(env, out, v, 11);
    }
    unmap_file(&m);
  }
  if (cl) (*env)->ReleaseIntArrayElements(env, contigs, cl, JNI_ABORT);
  free(bl);
}

/* loadBamIntervals' record pass over a shard (load/.../CanLoadBam.scala:120-154;
 * sbh_records_scan_regions): chunk flat ranges [chunkBegin[k], chunkEnd[k]) and the merged
 * intervals (ref, begin, end) 0-based half-open; out = {n, nameBytes, cigarOps, bases,
 * auxBytes} for recordsFetch. */
JNIEXPORT void JNICALL Java_org_hammerlab_bam_gpu_Native_00024_recordsScanRegions(
    JNIEnv *env, jobject self, jlong ctx, jlong sh, jlongArray chunkBegin, jlongArray chunkEnd, jintArray ivRef,
    jlongArray ivBegin, jlongArray ivEnd, jlongArray out) {
  const jsize nch = (*env)->GetArrayLength(env, chunkBegin), niv = (*env)->GetArrayLength(env, ivRef);
  if ((*env)->GetArrayLength(env, chunkEnd) != nch || (*env)->GetArrayLength(env, ivBegin) != niv ||
      (*env)->GetArrayLength(env, ivEnd) != niv) {
    throw_arg(env, "recordsScanRegions: arrays of different lengths");
    return;
  }
  uint64_t *cb = (uint64_t *)malloc(sizeof(uint64_t) * 2 * (size_t)(nch > 0 ? nch : 1));
  int64_t *iv = (int64_t *)malloc(sizeof(int64_t) * 2 * (size_t)(niv > 0 ? niv : 1));
  int32_t *ir = (int32_t *)malloc(sizeof(int32_t) * (size_t)(niv > 0 ? niv : 1));
  if (cb && iv && ir) {
    (*env)->GetLongArrayRegion(env, chunkBegin, 0, nch, (jlong *)cb);
    (*env)->GetLongArrayRegion(env, chunkEnd, 0, nch, (jlong *)(cb + nch));
    (*env)->GetLongArrayRegion(env, ivBegin, 0, niv, (jlong *)iv);
    (*env)->GetLongArrayRegion(env, ivEnd, 0, niv, (jlong *)(iv + niv));
    (*env)->GetIntArrayRegion(env, ivRef, 0, niv, (jint *)ir);
    sbh_records_sizes z;
    if (!failed(env, ctx, sbh_records_scan_regions(SH(sh), cb, cb + nch, (uint64_t)nch, ir, iv, iv + niv,
                                                   (uint32_t)niv, &z))) {
      jlong v[5] = {(jlong)z.n, (jlong)z.name_bytes, (jlong)z.cigar_ops, (jlong)z.bases, (jlong)z.aux_bytes};
      put_longs(env, out, v, 5);
    }
  } else {
    throw_status(env, NULL, SBH_E_NOMEM);
  }
  free(cb), free(iv), free(ir);
}
