// Native.scala -- the Scala side of jni/sparkbam_jni.c, and the façades a maintainer drops into
// spark-bam's modules so the hot path runs on libsparkbam_hip.so.  Signatures of the reference's
// own types are unchanged; only their bodies call Native.
//
//   check/src/main/scala/org/hammerlab/bam/check/Checker.scala:7-25    trait Checker / MakeChecker
//   check/src/main/scala/org/hammerlab/bam/check/eager/Checker.scala:165-177  eager MakeChecker implicit
//   load/src/main/scala/org/hammerlab/bam/spark/load/CanLoadBam.scala:196-357  loadSplitsAndReads et al.
package org.hammerlab.bam.gpu

import java.nio.ByteBuffer

class NeedHaloException(msg: String) extends RuntimeException(msg)

object Native {
  System.loadLibrary("sparkbam_jni")

  @native def ctxCreate(device: Int): Long
  @native def ctxDestroy(ctx: Long): Unit
  @native def hostAlloc(n: Long): ByteBuffer
  @native def hostFree(buf: ByteBuffer): Unit

  @native def shardCreate(ctx: Long, comp: ByteBuffer, n: Long, fileOffset: Long, fileSize: Long): Long
  @native def shardDestroy(sh: Long): Unit
  @native def findBlockStart(ctx: Long, sh: Long, start: Long, blocksToCheck: Int): Long
  @native def indexAndInflate(ctx: Long, sh: Long, start: Long, out: Array[Long]): Unit
  @native def blocks(ctx: Long, sh: Long, first: Long, count: Long, out: Array[Long]): Unit
  @native def readFlat(ctx: Long, sh: Long, flat: Long, n: Long, out: ByteBuffer): Unit
  @native def flatOf(ctx: Long, sh: Long, vpos: Long): Long
  @native def posOf(ctx: Long, sh: Long, flat: Long): Long
  @native def setContigs(ctx: Long, sh: Long, lengths: Array[Int]): Unit

  @native def checkEager(ctx: Long, sh: Long, begin: Long, end: Long, readsToCheck: Int, bits: ByteBuffer): Long
  @native def checkFull(ctx: Long, sh: Long, begin: Long, end: Long, readsToCheck: Int, words: ByteBuffer,
                        counts: ByteBuffer, rbe: ByteBuffer, closeFlat: ByteBuffer, closeWord: ByteBuffer,
                        closeCap: Long, out: Array[Long]): Unit
  @native def findRecordStart(ctx: Long, sh: Long, from: Long, readsToCheck: Int, maxReadSize: Int,
                              out: Array[Long]): Unit
  @native def chainFrom(ctx: Long, sh: Long, first: Long, endFlat: Long, out: Array[Long]): Unit
  @native def splitStarts(ctx: Long, sh: Long, starts: Array[Long], ends: Array[Long], blocksToCheck: Int,
                          readsToCheck: Int, maxReadSize: Int, out: Array[Long]): Unit
  @native def checkRecords(ctx: Long, sh: Long, ranges: Array[Long], readsToCheck: Int, recVpos: ByteBuffer,
                           nRec: Long, fpFlat: ByteBuffer, fnFlat: ByteBuffer, cap: Long, out: Array[Long]): Unit
  @native def runShard(ctx: Long, sh: Long, indexStart: Long, ownEnd: Long, readsToCheck: Int, maxReadSize: Int,
                       out: Array[Long]): Unit
  @native def runStream(ctx: Long, comp: ByteBuffer, n: Long, fileOffset: Long, fileSize: Long, indexStart: Long,
                        ownEnd: Long, window: Long, halo: Long, contigs: Array[Int], readsToCheck: Int,
                        maxReadSize: Int, out: Array[Long]): Unit
  @native def recordsScan(ctx: Long, sh: Long, first: Long, endFlat: Long, out: Array[Long]): Unit
  @native def recordsFetch(ctx: Long, sh: Long, columns: Array[ByteBuffer]): Unit
}

/** One executor GPU (one sbh_ctx), shared by its tasks under a lock (the reference's checkers are
  * single-threaded per task, PosChecker.scala:19-20). */
object Device {
  lazy val ctx: Long = Native.ctxCreate(sys.env.getOrElse("LOCAL_RANK", "0").toInt)
}

/** A split's compressed bytes + halo, resident in HBM, indexed and inflated from `start`. */
class GpuShard(comp: ByteBuffer, n: Long, fileOffset: Long, fileSize: Long, contigs: Array[Int])
  extends AutoCloseable {
  private val ctx = Device.ctx
  val sh: Long = Native.shardCreate(ctx, comp, n, fileOffset, fileSize)
  Native.setContigs(ctx, sh, contigs)
  private val nf = new Array[Long](2)
  def load(start: Long): Unit = Native.indexAndInflate(ctx, sh, start, nf)
  def flatSize: Long = nf(1)
  def flatOf(vpos: Long): Long = Native.flatOf(ctx, sh, vpos)
  def eagerBits(readsToCheck: Int): ByteBuffer = {
    val bits = ByteBuffer.allocateDirect(((flatSize + 7) / 8).toInt)
    Native.checkEager(ctx, sh, 0, flatSize, readsToCheck, bits)
    bits
  }
  /** (status, firstVpos, count) per split, one batch (CanLoadBam.scala:283-297, 316-356). */
  def splits(starts: Array[Long], ends: Array[Long], blocksToCheck: Int, readsToCheck: Int,
             maxReadSize: Int): Array[(Int, Long, Long)] = {
    val out = new Array[Long](3 * starts.length)
    Native.splitStarts(ctx, sh, starts, ends, blocksToCheck, readsToCheck, maxReadSize, out)
    Array.tabulate(starts.length)(i => (out(3 * i).toInt, out(3 * i + 1), out(3 * i + 2)))
  }
  override def close(): Unit = Native.shardDestroy(sh)
}

/** Drop-in for check/.../eager/Checker.scala: the same trait, answered from one batched call.
  * (In the reference build this extends org.hammerlab.bam.check.Checker[Boolean] and takes
  * the implicit ReadsToCheck / ContigLengths the eager MakeChecker passes, eager/Checker.scala:165-177.) */
class EagerChecker(shard: GpuShard, readsToCheck: Int) {
  private lazy val bits = shard.eagerBits(readsToCheck)
  def apply(vpos: Long): Boolean = {
    val f = shard.flatOf(vpos)
    (bits.get((f >> 3).toInt) & (1 << (f & 7).toInt)) != 0
  }
}
