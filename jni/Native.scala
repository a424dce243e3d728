// Native.scala -- the Scala side of jni/sparkbam_jni.c, and the façades a maintainer drops into
// spark-bam's modules so the hot path runs on libsparkbam_hip.so.  Each façade implements the
// reference's own trait with the reference's own signature; only the bodies call Native.
//
//   check/src/main/scala/org/hammerlab/bam/check/Checker.scala:7-25          Checker[+Call], MakeChecker
//   check/src/main/scala/org/hammerlab/bam/check/ReadStartFinder.scala:5-11  ReadStartFinder.nextReadStart
//   check/src/main/scala/org/hammerlab/bam/check/eager/Checker.scala:165-177 eager makeChecker implicit
//   check/src/main/scala/org/hammerlab/bam/check/full/Checker.scala:186-198  full makeChecker implicit
//   check/src/main/scala/org/hammerlab/bam/check/full/error/Flags.scala:10-45 Result / Success / Flags
//   bgzf/src/main/scala/org/hammerlab/bgzf/block/Stream.scala:16-75          StreamI (Block iterator)
//   load/src/main/scala/org/hammerlab/bam/spark/load/CanLoadBam.scala:196-357 loadSplitsAndReads et al.
//
// Not compiled in this image (no JVM / sbt; SURVEY.md 8c); the C-ABI under it is the tested
// contract (tests/test_abi.py, every -m gpu test calls it).
package org.hammerlab.bam.gpu

import java.nio.{ ByteBuffer, ByteOrder }

import org.apache.spark.broadcast.Broadcast
import org.hammerlab.bam.check.Checker.MakeChecker
import org.hammerlab.bam.check.{ Checker, MaxReadSize, ReadStartFinder, ReadsToCheck }
import org.hammerlab.bam.check.full.error.{ Flags, Result, Success }
import org.hammerlab.bam.header.ContigLengths
import org.hammerlab.bgzf.Pos
import org.hammerlab.bgzf.block.{ Block, StreamI }
import org.hammerlab.channel.{ ByteChannel, CachingChannel, SeekableByteChannel }

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
  @native def eagerBits(ctx: Long, sh: Long, begin: Long, end: Long, bits: ByteBuffer): Unit
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
  /** sbh_run_stream2: per-split (status, firstVpos, count) into splitOut (3 longs per split) and
    * out = {nWindows, compBytes, flatBytes, nTrue, count, firstVpos, exitVpos, crcBadBlocks}. */
  @native def runStreamSplits(ctx: Long, comp: ByteBuffer, n: Long, fileOffset: Long, fileSize: Long,
                              indexStart: Long, ownEnd: Long, window: Long, halo: Long, contigs: Array[Int],
                              blocksToCheck: Int, readsToCheck: Int, maxReadSize: Int, verifyCrc: Boolean,
                              splitStarts: Array[Long], splitEnds: Array[Long], splitOut: Array[Long],
                              out: Array[Long]): Unit
  /** out = {nRecords, nameBytes, cigarOps, bases, auxBytes} */
  @native def recordsScan(ctx: Long, sh: Long, first: Long, endFlat: Long, out: Array[Long]): Unit
  /** 18 direct buffers in sbh_records_out order, sized from recordsScan's `sizes` */
  @native def recordsFetch(ctx: Long, sh: Long, sizes: Array[Long], columns: Array[ByteBuffer]): Unit
  /** htsjdk-rewrite's BGZF writer (sbh_bgzf_compress_level; level 5 = htsjdk's bytes):
    * returns the file length written into `out` (capacity >= bgzfBound(n)). */
  @native def bgzfBound(n: Long): Long
  @native def bgzfCompress(ctx: Long, src: ByteBuffer, n: Long, level: Int, out: ByteBuffer): Long
}

/** One executor GPU (one sbh_ctx), shared by its tasks under a lock (the reference's checkers are
  * single-threaded per task, PosChecker.scala:19-20). */
object Device {
  lazy val ctx: Long = Native.ctxCreate(sys.env.getOrElse("LOCAL_RANK", "0").toInt)
}

/** Compressed bytes [fileOffset, fileOffset + n) of a BGZF file, resident in HBM, indexed and
  * inflated from block `start`, with the eager bitmap of every position once asked for. */
class GpuShard(comp: ByteBuffer, n: Long, val fileOffset: Long, fileSize: Long, contigs: Array[Int])
  extends AutoCloseable {
  private val ctx = Device.ctx
  val sh: Long = Native.shardCreate(ctx, comp, n, fileOffset, fileSize)
  Native.setContigs(ctx, sh, contigs)
  private val nf = new Array[Long](2)
  def load(start: Long): Unit = Native.indexAndInflate(ctx, sh, start, nf)
  def numBlocks: Long = nf(0)
  def flatSize: Long = nf(1)
  def flatOf(pos: Pos): Long = Native.flatOf(ctx, sh, pos.toHTSJDK)
  def posOf(flat: Long): Pos = Pos(Native.posOf(ctx, sh, flat))
  /** (start, ustart, csize, hsize, usize, flags) of blocks [first, first + count) */
  def blocks(first: Long, count: Long): Array[Long] = {
    val out = new Array[Long](6 * count.toInt)
    Native.blocks(ctx, sh, first, count, out)
    out
  }
  def flat(from: Long, n: Int): Array[Byte] = {
    val b = ByteBuffer.allocateDirect(n)
    Native.readFlat(ctx, sh, from, n, b)
    val a = new Array[Byte](n)
    b.get(a)
    a
  }

  private var bits: ByteBuffer = _
  def eagerBits(readsToCheck: Int): ByteBuffer = {
    if (bits == null) {
      bits = ByteBuffer.allocateDirect(((flatSize + 7) / 8).toInt)
      Native.checkEager(ctx, sh, 0, flatSize, readsToCheck, bits)
    }
    bits
  }
  def fullWord(flat: Long, readsToCheck: Int): Int = {
    val w = ByteBuffer.allocateDirect(4).order(ByteOrder.LITTLE_ENDIAN)
    val out = new Array[Long](2)
    Native.checkFull(ctx, sh, flat, flat + 1, readsToCheck, w, null, null, null, null, 0, out)
    w.getInt(0)
  }
  def findRecordStart(from: Long, readsToCheck: Int, maxReadSize: Int): Option[(Long, Int)] = {
    val out = new Array[Long](2)
    try {
      Native.findRecordStart(ctx, sh, from, readsToCheck, maxReadSize, out)
      Some((out(0), out(1).toInt))
    } catch {
      case _: org.hammerlab.bam.check.NoReadFoundException ⇒ None
    }
  }
  /** (status, firstVpos, count) per split, one batch (CanLoadBam.scala:283-297, 316-356). */
  def splits(starts: Array[Long], ends: Array[Long], blocksToCheck: Int, readsToCheck: Int,
             maxReadSize: Int): Array[(Int, Long, Long)] = {
    val out = new Array[Long](3 * starts.length)
    Native.splitStarts(ctx, sh, starts, ends, blocksToCheck, readsToCheck, maxReadSize, out)
    Array.tabulate(starts.length)(i ⇒ (out(3 * i).toInt, out(3 * i + 1), out(3 * i + 2)))
  }
  override def close(): Unit = Native.shardDestroy(sh)
}

object GpuShard {
  val Halo: Long = 4L << 20

  /** The window [lo, lo + window) of the channel's file plus a halo, indexed from the first
    * block at/after lo (FindBlockStart, bgzf/.../block/FindBlockStart.scala:8-36) and inflated. */
  def load(ch: CachingChannel[SeekableByteChannel], lo: Long, window: Long, contigs: Array[Int],
           blocksToCheck: Int = 5): GpuShard = {
    val size = ch.size
    val n = math.min(size - lo, window + Halo)
    val buf = Native.hostAlloc(n)
    ch.seek(lo)
    ch.readFully(buf)
    buf.flip()
    val s = new GpuShard(buf, n, lo, size, contigs)
    s.load(Native.findBlockStart(Device.ctx, s.sh, lo, blocksToCheck))
    Native.hostFree(buf)
    s
  }

  def contigArray(contigLengths: ContigLengths): Array[Int] =
    contigLengths.map.values.map(_._2.toInt).toArray
}

/** Drop-in for check/.../eager/Checker.scala: Checker[Boolean] with ReadStartFinder, answered
  * from the eager bitmap of a GPU window that holds the asked position (the window slides
  * when a position past it is asked; a partition's positions come in order,
  * CallPartition.scala:35-52). */
class GpuEagerChecker(ch: CachingChannel[SeekableByteChannel],
                      contigLengths: ContigLengths,
                      readsToCheck: ReadsToCheck,
                      window: Long = 256L << 20)
  extends Checker[Boolean]
    with ReadStartFinder {

  private val contigs = GpuShard.contigArray(contigLengths)
  private var shard: GpuShard = _
  private var hi = -1L  // first file offset past the window's owned blocks

  private def shardFor(blockPos: Long): GpuShard = {
    if (shard == null || blockPos < shard.fileOffset || blockPos >= hi) {
      if (shard != null) shard.close()
      shard = GpuShard.load(ch, blockPos, window, contigs)
      hi = blockPos + window
    }
    shard
  }

  override def apply(pos: Pos): Boolean = {
    val s = shardFor(pos.blockPos)
    val f = s.flatOf(pos)
    val bits = s.eagerBits(readsToCheck.n)
    (bits.get((f >> 3).toInt) & (1 << (f & 7).toInt)) != 0
  }

  override def nextReadStart(start: Pos)(implicit maxReadSize: MaxReadSize): Option[Pos] = {
    val s = shardFor(start.blockPos)
    s.findRecordStart(s.flatOf(start), readsToCheck.n, maxReadSize.n).map { case (f, _) ⇒ s.posOf(f) }
  }
}

object GpuEagerChecker {
  /** The eager checker's MakeChecker (eager/Checker.scala:165-177), GPU-backed. */
  implicit def makeChecker(implicit
                           contigLengths: Broadcast[ContigLengths],
                           readsToCheck: ReadsToCheck): MakeChecker[Boolean, GpuEagerChecker] =
    new MakeChecker[Boolean, GpuEagerChecker] {
      override def apply(ch: CachingChannel[SeekableByteChannel]): GpuEagerChecker =
        new GpuEagerChecker(ch, contigLengths.value, readsToCheck)
    }
}

/** Drop-in for check/.../full/Checker.scala: Checker[Result] -- the GPU's full-checker word
  * (include/sparkbam.h: bit 31 Success, bits 20-29 readsParsed / readsBeforeError, bits 0-18
  * the Flags in Flags.scala's serde order) turned back into Success(n) or Flags(...). */
class GpuFullChecker(ch: CachingChannel[SeekableByteChannel],
                     contigLengths: ContigLengths,
                     readsToCheck: ReadsToCheck,
                     window: Long = 256L << 20)
  extends Checker[Result] {

  private val contigs = GpuShard.contigArray(contigLengths)
  private var shard: GpuShard = _
  private var hi = -1L

  override def apply(pos: Pos): Result = {
    if (shard == null || pos.blockPos < shard.fileOffset || pos.blockPos >= hi) {
      if (shard != null) shard.close()
      shard = GpuShard.load(ch, pos.blockPos, window, contigs)
      hi = pos.blockPos + window
    }
    GpuFullChecker.result(shard.fullWord(shard.flatOf(pos), readsToCheck.n))
  }
}

object GpuFullChecker {
  def result(w: Int): Result = {
    val n = (w >>> 20) & 0x3ff
    if ((w & 0x80000000) != 0) Success(n)
    else {
      def b(i: Int) = (w & (1 << i)) != 0
      Flags(b(0), b(1), b(2), b(3), b(4), b(5), b(6), b(7), b(8), b(9), b(10), b(11), b(12), b(13), b(14), b(15),
            b(16), b(17), b(18), n)
    }
  }

  /** The full checker's MakeChecker (full/Checker.scala:186-198), GPU-backed. */
  implicit def makeChecker(implicit
                           contigLengths: Broadcast[ContigLengths],
                           readsToCheck: ReadsToCheck): MakeChecker[Result, GpuFullChecker] =
    new MakeChecker[Result, GpuFullChecker] {
      override def apply(ch: CachingChannel[SeekableByteChannel]): GpuFullChecker =
        new GpuFullChecker(ch, contigLengths.value, readsToCheck)
    }
}

/** Drop-in for bgzf/.../block/Stream.scala's StreamI: the Block iterator over a channel, blocks
  * inflated on the GPU a window at a time; Block.bytes is copied out only for the block handed
  * out (Block.scala:12-46).  An empty block ends the stream (Stream.scala:56-58). */
case class GpuStream(compressedBytes: ByteChannel with SeekableByteChannel, window: Long = 256L << 20)
  extends StreamI {

  private var shard: GpuShard = _
  private var table: Array[Long] = Array.empty
  private var next = 0L  // next block of the window's table
  private var lo = compressedBytes.position()

  private def refill(): Boolean = {
    if (shard != null) shard.close()
    if (lo >= compressedBytes.size) return false
    val n = math.min(compressedBytes.size - lo, window + GpuShard.Halo)
    val buf = Native.hostAlloc(n)
    compressedBytes.seek(lo)
    compressedBytes.readFully(buf)
    buf.flip()
    shard = new GpuShard(buf, n, lo, compressedBytes.size, Array.empty[Int])
    shard.load(lo)
    Native.hostFree(buf)
    table = shard.blocks(0, shard.numBlocks)
    next = 0
    true
  }

  override protected def _advance: Option[Block] = {
    if (shard == null || next >= shard.numBlocks || table(6 * next.toInt) >= lo + window) {
      if (shard != null && next < shard.numBlocks) lo = table(6 * next.toInt)
      if (!refill()) return None
    }
    val i = 6 * next.toInt
    val (start, ustart, csize, usize, flags) = (table(i), table(i + 1), table(i + 2), table(i + 4), table(i + 5))
    if ((flags & 1) != 0) return None  // an empty block ends the stream
    next += 1
    lo = start + csize
    Some(Block(shard.flat(ustart, usize.toInt), start, csize.toInt))
  }
}
