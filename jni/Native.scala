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
import hammerlab.path._

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
  @native def flatBound(ctx: Long, sh: Long, fileOff: Long): Long
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

/** Compressed bytes [fileOffset, fileOffset + n) of a BGZF file, resident in HBM. */
class GpuShard(comp: ByteBuffer, n: Long, val fileOffset: Long, fileSize: Long, contigs: Array[Int])
  extends AutoCloseable {
  private val ctx = Device.ctx
  val sh: Long = Native.shardCreate(ctx, comp, n, fileOffset, fileSize)
  Native.setContigs(ctx, sh, contigs)
  val atEof: Boolean = fileOffset + n == fileSize
  private val nf = new Array[Long](2)
  def load(start: Long): Unit = Native.indexAndInflate(ctx, sh, start, nf)
  def numBlocks: Long = nf(0)
  def flatSize: Long = nf(1)
  def flatOf(pos: Pos): Long = Native.flatOf(ctx, sh, pos.toHTSJDK)
  def posOf(flat: Long): Pos = Pos(Native.posOf(ctx, sh, flat))
  /** flat image of Pos(fileOff, 0) as an exclusive bound (sbh_flat_bound) */
  def flatBound(fileOff: Long): Long = Native.flatBound(ctx, sh, fileOff)
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
  /** the eager bit of every flat position of [begin, end), in one batch */
  def eagerBits(begin: Long, end: Long, readsToCheck: Int): ByteBuffer = {
    val bits = ByteBuffer.allocateDirect(math.max(1L, (end - begin + 7) / 8).toInt)
    Native.checkEager(ctx, sh, begin, end, readsToCheck, bits)
    bits
  }
  /** the full-checker word of every flat position of [begin, end), in one batch */
  def fullWords(begin: Long, end: Long, readsToCheck: Int): ByteBuffer = {
    val words = ByteBuffer.allocateDirect(math.max(4L, 4 * (end - begin)).toInt).order(ByteOrder.LITTLE_ENDIAN)
    Native.checkFull(ctx, sh, begin, end, readsToCheck, words, null, null, null, null, 0, new Array[Long](2))
    words
  }
  /** FindRecordStart.withDelta from a flat position: Some((flat, delta)) or None */
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
  /** [lo, min(size, lo + n)) of the channel's file as a resident shard */
  def read(ch: SeekableByteChannel, lo: Long, n: Long, contigs: Array[Int]): GpuShard = {
    val size = ch.size
    val m = math.min(size - lo, n)
    val buf = Native.hostAlloc(m)
    try {
      ch.seek(lo)
      ch.readFully(buf)
      buf.flip()
      new GpuShard(buf, m, lo, size, contigs)
    } finally Native.hostFree(buf)
  }

  def contigArray(contigLengths: ContigLengths): Array[Int] =
    contigLengths.map.values.map(_._2.toInt).toArray
}

/** A window of the file on the GPU: compressed bytes [lo, lo + window + halo) indexed from
  * FindBlockStart(lo) (bgzf/.../block/FindBlockStart.scala:8-36) and inflated.  It owns the blocks
  * starting in [lo, hi = lo + window), i.e. flat positions [0, owned = flatBound(hi)); the halo
  * only feeds the chains of the owned positions.  A halo with no block past hi throws
  * NeedHaloException (the last owned block, or what follows it, is cut off).  Mirrored by
  * spark_bam_amd.checkers.GpuWindow. */
class GpuWindow(val shard: GpuShard, val lo: Long, val hi: Long) extends AutoCloseable {
  val atEof: Boolean = shard.atEof
  val owned: Long = shard.flatBound(hi)
  if (!atEof && owned == shard.flatSize) {
    shard.close()
    throw new NeedHaloException(s"no block past $hi in the halo")
  }
  // the host block table: flatOf(pos) without a JNI call per position
  private val table = shard.blocks(0, shard.numBlocks)
  private val starts = Array.tabulate(shard.numBlocks.toInt)(i ⇒ table(6 * i))
  def owns(blockPos: Long): Boolean = lo <= blockPos && blockPos < hi
  def flatOf(pos: Pos): Long = {
    val i = java.util.Arrays.binarySearch(starts, pos.blockPos)
    if (i < 0) throw new IllegalArgumentException(s"${pos.blockPos} is not a block start of this window")
    table(6 * i + 1) + pos.offset
  }
  def posOf(flat: Long): Pos = shard.posOf(flat)
  override def close(): Unit = shard.close()
}

object GpuWindow {
  def load(ch: SeekableByteChannel, lo: Long, window: Long, halo: Long, contigs: Array[Int],
           blocksToCheck: Int): GpuWindow = {
    val s = GpuShard.read(ch, lo, window + halo, contigs)
    try {
      s.load(Native.findBlockStart(Device.ctx, s.sh, lo, blocksToCheck))
    } catch {
      case e: Throwable ⇒ s.close(); throw e
    }
    new GpuWindow(s, lo, lo + window)
  }
}

/** The window cache both checkers share: the window holding the asked block (a partition's
  * positions come in order, CallPartition.scala:35-52, so a window serves a run of calls) plus
  * its batch (`fill`), reloaded with 4x the halo whenever either needs bytes past it. */
abstract class WindowedChecker[B](ch: SeekableByteChannel, contigs: Array[Int], val readsToCheck: Int,
                                  window: Long, var halo: Long, blocksToCheck: Int) {
  protected def fill(w: GpuWindow): B

  protected var w: GpuWindow = _
  protected var batch: B = _

  private def load(lo: Long): Unit = {
    while (true) {
      var nw: GpuWindow = null
      try {
        nw = GpuWindow.load(ch, lo, window, halo, contigs, blocksToCheck)
        batch = fill(nw)
        w = nw
        return
      } catch {
        case e: NeedHaloException ⇒
          if (nw != null) nw.close()
          if (lo + window + halo >= ch.size) throw e
          halo *= 4
      }
    }
  }

  protected def windowFor(blockPos: Long, reload: Boolean = false): GpuWindow = {
    if (reload || w == null || !w.owns(blockPos)) {
      if (w != null) { w.close(); w = null }
      load(blockPos)
    }
    w
  }

  def close(): Unit = if (w != null) { w.close(); w = null }
}

/** Drop-in for check/.../eager/Checker.scala: Checker[Boolean] with ReadStartFinder.  apply(pos)
  * is a lookup in the window's eager bitmap, computed over the OWNED positions only
  * ([0, flatBound(hi)): no position whose answer needs bytes past the halo); nextReadStart is
  * FindRecordStart on the device, the halo grown on NeedHaloException.  Mirrored call for call by
  * spark_bam_amd.checkers.WindowedEagerChecker (tests/test_checkers_gpu.py). */
class GpuEagerChecker(ch: SeekableByteChannel,
                      contigLengths: ContigLengths,
                      readsToCheck: ReadsToCheck,
                      window: Long = 256L << 20,
                      halo: Long = 4L << 20,
                      blocksToCheck: Int = 5)
  extends WindowedChecker[ByteBuffer](ch, GpuShard.contigArray(contigLengths), readsToCheck.n, window, halo,
                                      blocksToCheck)
    with Checker[Boolean]
    with ReadStartFinder {

  override protected def fill(w: GpuWindow): ByteBuffer = w.shard.eagerBits(0, w.owned, readsToCheck.n)

  override def apply(pos: Pos): Boolean = {
    val f = windowFor(pos.blockPos).flatOf(pos)
    (batch.get((f >> 3).toInt) & (1 << (f & 7).toInt)) != 0
  }

  override def nextReadStart(start: Pos)(implicit maxReadSize: MaxReadSize): Option[Pos] = {
    var reload = false
    while (true) {
      val cur = windowFor(start.blockPos, reload)
      try {
        return cur.shard.findRecordStart(cur.flatOf(start), readsToCheck.n, maxReadSize.n).map {
          case (f, _) ⇒ cur.posOf(f)
        }
      } catch {
        case e: NeedHaloException ⇒
          if (cur.atEof) throw e
          halo *= 4
          reload = true
      }
    }
    None
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

/** Drop-in for check/.../full/Checker.scala: Checker[Result].  The window's full-checker words
  * (include/sparkbam.h: bit 31 Success, bits 20-29 readsParsed / readsBeforeError, bits 0-18 the
  * Flags in Flags.scala's serde order) are computed once per window over its owned positions;
  * apply(pos) turns one back into Success(n) or Flags(...).  32 MiB windows keep the word buffer
  * (4 B per position) near 400 MB.  Mirrored by spark_bam_amd.checkers.WindowedFullChecker. */
class GpuFullChecker(ch: SeekableByteChannel,
                     contigLengths: ContigLengths,
                     readsToCheck: ReadsToCheck,
                     window: Long = 32L << 20,
                     halo: Long = 4L << 20,
                     blocksToCheck: Int = 5)
  extends WindowedChecker[ByteBuffer](ch, GpuShard.contigArray(contigLengths), readsToCheck.n, window, halo,
                                      blocksToCheck)
    with Checker[Result] {

  override protected def fill(w: GpuWindow): ByteBuffer = w.shard.fullWords(0, w.owned, readsToCheck.n)

  override def apply(pos: Pos): Result = {
    val f = windowFor(pos.blockPos).flatOf(pos)
    GpuFullChecker.result(batch.getInt((4 * f).toInt))
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

/** Drop-in for load/.../CanLoadBam.scala:268-302,316-356 (loadSplitsAndReads / loadBam's splits
  * and per-partition counts) on the executors' GPUs.  The Hadoop FileSplits (SPLIT_SLOP 1.1,
  * FileSplits.asJava) are dealt to `numTasks` Spark tasks as contiguous runs; each task loads its
  * byte range plus a halo into one shard and runs FindBlockStart + index + inflate + the eager
  * check at every owned position + every split's FindRecordStart and record count in a few
  * launches (runTask); the driver collects the TaskParts, forms the splits by sliding2 over the
  * non-empty splits' first records with Pos(fileSize, 0), and checks that the record chain leaving
  * each task enters the next non-empty task at its first record, re-walking that task from the
  * upstream exit (rewalk, a task of its own) where it does not.  Record decoding stays htsjdk's
  * (loadBam: RecordStream from each split's first record while pos < the split's end).
  * Mirrored call for call by spark_bam_amd.sharded.load_splits_and_reads_tasks / RankRun
  * (tests/test_sharded.py test_gpu_tasks_*). */
object GpuLoadBam {
  /** One task's answer: per split (first record vpos or -1, count), and the task's record chain
    * (first vpos or -1, count, exit vpos or -1: the first chain record at/after the task's end). */
  case class TaskPart(task: Int, splitIndex: Int, firsts: Array[Long], counts: Array[Long], first: Long, count: Long,
                      exit: Long)

  /** Hadoop FileInputFormat.getSplits' arithmetic (SPLIT_SLOP 1.1) */
  def fileSplits(size: Long, splitSize: Long): Array[(Long, Long)] = {
    val out = scala.collection.mutable.ArrayBuffer[(Long, Long)]()
    var rem = size
    while (rem.toDouble / splitSize > 1.1) { out += ((size - rem, size - rem + splitSize)); rem -= splitSize }
    if (rem != 0) out += ((size - rem, size))
    out.toArray
  }

  /** task t's contiguous run of splits: (index of its first split, its splits) */
  def taskSplits(size: Long, splitSize: Long, tasks: Int, t: Int): (Int, Array[(Long, Long)]) = {
    val all = fileSplits(size, splitSize)
    val a = t * all.length / tasks
    (a, all.slice(a, (t + 1) * all.length / tasks))
  }

  private def exitVpos(s: GpuShard, flat: Long): Long = try s.posOf(flat).toHTSJDK catch { case _: Exception ⇒ -1L }

  def runTask(path: Path, t: Int, splitIndex: Int, splits: Array[(Long, Long)], contigs: Array[Int],
              halo0: Long = 1L << 20, blocksToCheck: Int = 5, readsToCheck: Int = 10,
              maxReadSize: Int = 100000000): TaskPart = {
    if (splits.isEmpty) return TaskPart(t, splitIndex, Array.empty, Array.empty, -1L, 0L, -1L)
    val ch = SeekableByteChannel(path)
    try {
      val (lo, hi) = (splits.head._1, splits.last._2)
      var halo = halo0
      while (true) {
        val s = GpuShard.read(ch, lo, hi - lo + halo, contigs)
        try {
          val start = Native.findBlockStart(Device.ctx, s.sh, lo, blocksToCheck)
          val r = new Array[Long](7)  // nBlocks, compBytes, flatBytes, nTrue, firstVpos, count, exitFlat
          Native.runShard(Device.ctx, s.sh, start, hi, readsToCheck, maxReadSize, r)
          val per = s.splits(splits.map(_._1), splits.map(_._2), blocksToCheck, readsToCheck, maxReadSize)
          per.zip(splits).find(_._1._1 != 0).foreach {
            case ((st, _, _), (a, e)) ⇒ throw new IllegalStateException(s"split $a-$e: status $st")
          }
          val exit = if (r(5) > 0) exitVpos(s, r(6)) else -1L
          return TaskPart(t, splitIndex, per.map { case (_, v, n) ⇒ if (n > 0) v else -1L }, per.map(_._3),
                          if (r(5) > 0) r(4) else -1L, r(5), exit)
        } catch {
          case e: NeedHaloException ⇒
            if (hi + halo >= ch.size) throw e
            halo *= 4
        } finally s.close()
      }
      throw new IllegalStateException("unreachable")
    } finally ch.close()
  }

  /** The chain from fromVpos through the task's range [.., hi), window by window (each window's
    * eager bitmap first, then the chain): (records, exit vpos or -1). */
  def rewalk(path: Path, hi: Long, halo0: Long, contigs: Array[Int], fromVpos: Long, readsToCheck: Int = 10,
             window: Long = 1L << 30): (Long, Long) = {
    val ch = SeekableByteChannel(path)
    try {
      var total = 0L
      var v = fromVpos
      while (true) {
        val blo = v >>> 16
        if (blo >= hi) return (total, v)
        val whi = math.min(hi, blo + window)
        var halo = math.max(halo0, 1L << 20)
        var (n, ex, nxt) = (0L, -1L, -1L)
        var done = false
        while (!done) {
          val s = GpuShard.read(ch, blo, whi - blo + halo, contigs)
          try {
            s.load(blo)
            val f = s.flatOf(Pos(v))
            val e = s.flatBound(whi)
            Native.checkEager(Device.ctx, s.sh, f, e, readsToCheck, null)
            val out = new Array[Long](2)
            Native.chainFrom(Device.ctx, s.sh, f, e, out)
            n = out(0)
            ex = if (n > 0) exitVpos(s, out(1)) else v
            val t = s.blocks(0, s.numBlocks)
            nxt = (0 until s.numBlocks.toInt).map(i ⇒ t(6 * i)).find(_ >= whi).getOrElse(-1L)
            done = true
          } catch {
            case e: NeedHaloException ⇒
              if (whi + halo >= ch.size) throw e
              halo *= 4
          } finally s.close()
        }
        total += n
        if (ex < 0 || whi >= hi) return (total, ex)
        v = if (ex == v) { if (nxt < 0) throw new NeedHaloException(s"no block past $whi"); nxt << 16 } else ex
      }
      (total, v)
    } finally ch.close()
  }

  /** Chain mismatches of the non-empty tasks in order: (next task, upstream exit vpos) where the
    * chain leaving a task does not enter the next one at its first record (after re-walks). */
  def mismatches(parts: Seq[TaskPart], rewalks: Map[Int, (Long, Long, Long)]): Seq[(Int, Long)] = {
    val eff = parts.map(p ⇒ rewalks.get(p.task).map { case (f, n, x) ⇒ (p.task, f, n, x) }
                                  .getOrElse((p.task, p.first, p.count, p.exit))).filter(_._3 > 0)
    eff.zip(eff.drop(1)).collect { case (a, b) if a._4 != b._2 && a._4 >= 0 ⇒ (b._1, a._4) }
  }

  /** loadSplitsAndReads' splits and per-split record counts (CanLoadBam.scala:268-302). */
  def loadSplitsAndCounts(sc: org.apache.spark.SparkContext, path: Path, splitSize: Long, numTasks: Int,
                          contigLengths: ContigLengths): (Vector[org.hammerlab.bam.spark.Split], Vector[Long]) = {
    val size = path.size
    val contigs = GpuShard.contigArray(contigLengths)
    val tasks = (0 until numTasks).map(t ⇒ (t, taskSplits(size, splitSize, numTasks, t)))
    val parts = sc.parallelize(tasks, numTasks)
      .map { case (t, (a, sp)) ⇒ runTask(path, t, a, sp, contigs) }
      .collect()
      .sortBy(_.splitIndex)
      .toSeq
    var rewalks = Map.empty[Int, (Long, Long, Long)]
    var round = 0
    var todo = mismatches(parts, rewalks)
    while (todo.nonEmpty && round < numTasks) {
      val his = parts.map(p ⇒ p.task → (if (p.counts.isEmpty) 0L else taskSplits(size, splitSize, numTasks, p.task)._2.last._2)).toMap
      val redone = sc.parallelize(todo.distinct, todo.size)
        .map { case (t, v) ⇒ t → { val (n, x) = rewalk(path, his(t), 1L << 20, contigs, v); (v, n, x) } }
        .collect()
      rewalks ++= redone
      todo = mismatches(parts, rewalks)
      round += 1
    }
    val firsts = parts.flatMap(p ⇒ p.firsts.zip(p.counts).collect { case (v, n) if n > 0 ⇒ Pos(v) })
    val splits = firsts.zip(firsts.drop(1) :+ Pos(size, 0)).map { case (a, b) ⇒ org.hammerlab.bam.spark.Split(a, b) }
    (splits.toVector, parts.flatMap(_.counts).toVector)
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
    shard = GpuShard.read(compressedBytes, lo, window + (4L << 20), Array.empty[Int])
    shard.load(lo)
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
