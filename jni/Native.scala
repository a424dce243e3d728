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
//   load/src/main/scala/org/hammerlab/bam/spark/load/CanLoadBam.scala:61-405  loadBam / loadSplitsAndReads /
//                                                                            loadReadsAndPositions / loadReads /
//                                                                            loadBamIntervals (GpuCanLoadBam)
//   check/src/main/scala/org/hammerlab/bam/spark/FindRecordStart.scala:11-71  FindRecordStart, NoReadFoundException
//   bgzf/src/main/scala/org/hammerlab/bgzf/block/FindBlockStart.scala:8-36  FindBlockStart, HeaderSearchFailedException
//   check/src/main/scala/org/hammerlab/bam/check/Blocks.scala:141-206       Blocks.apply's unindexed branch (GpuBlocks)
//
// Not compiled in this image (no JVM / sbt; SURVEY.md 8c); the C-ABI under it is the tested
// contract (tests/test_abi.py, every -m gpu test calls it), and the reference names this file
// and the shim use -- classes, constructors, imports, overridden signatures -- are pinned
// against the reference's own declarations by tests/test_jni_names.py.
package org.hammerlab.bam.gpu

import java.nio.{ ByteBuffer, ByteOrder }

import hammerlab.iterator._
import hammerlab.path._
import htsjdk.samtools.{ DefaultSAMRecordFactory, SAMFileHeader, SAMRecord }
import org.apache.spark.broadcast.Broadcast
import org.apache.spark.rdd.RDD
import org.hammerlab.bam.check.Checker.{ MakeChecker, default }
import org.hammerlab.bam.check.{ Checker, MaxReadSize, ReadStartFinder, ReadsToCheck }
import org.hammerlab.bam.check.full.error.{ Flags, Result, Success }
import org.hammerlab.bam.header.{ ContigLengths, Header }
import org.hammerlab.bam.index.Index.Chunk
import org.hammerlab.bam.spark.{ BAMRecordRDD, NoReadFoundException, Split }
import org.hammerlab.bam.spark.load.{ CanLoadBam, SplitRDD }
import org.hammerlab.bgzf.{ EstimatedCompressionRatio, Pos }
import org.hammerlab.bgzf.block.{ BGZFBlocksToCheck, Block, HeaderSearchFailedException, Metadata, SeekableStream,
                                   SeekableUncompressedBytes, StreamI }
import org.hammerlab.channel.{ ByteChannel, CachingChannel, SeekableByteChannel }
import org.hammerlab.genomics.loci.set.LociSet
import org.hammerlab.hadoop.splits.{ FileSplits, MaxSplitSize }

import scala.collection.JavaConverters._

class NeedHaloException(msg: String) extends RuntimeException(msg)

/** A library status the shim cannot turn into the reference's exception by itself: the
  * reference class needs the file's Path, which only the Scala caller holds.  `fields` are
  * sbh_last_error_detail's (include/sparkbam.h); Native.rethrow(path) builds the reference's
  * exception from them. */
class NativeException(val status: Int, msg: String, val fields: Array[Long]) extends RuntimeException(msg)

object Native {
  System.loadLibrary("sparkbam_jni")

  // include/sparkbam.h status codes the facades test for
  val HEADER_SEARCH_FAILED = 11
  val NO_READ_FOUND = 16
  val NOT_FOUND = 19
  val BAD_RECORD = 20

  /** The reference's exception for a NativeException, given the file's path:
    * HeaderSearchFailedException(path, start, positionsAttempted) (bgzf/.../block/
    * HeaderSearchFailedException.scala:7-12) or NoReadFoundException(path, start, maxReadSize)
    * (check/.../spark/FindRecordStart.scala:66-71). */
  def rethrow[T](path: Path): PartialFunction[Throwable, T] = {
    case e: NativeException if e.status == HEADER_SEARCH_FAILED ⇒
      throw HeaderSearchFailedException(path, e.fields(0), e.fields(1).toInt)
    case e: NativeException if e.status == NO_READ_FOUND ⇒
      throw NoReadFoundException(path, e.fields(0), e.fields(1).toInt)
  }

  @native def ctxCreate(device: Int): Long
  @native def ctxDestroy(ctx: Long): Unit
  @native def hostAlloc(n: Long): ByteBuffer
  @native def hostFree(buf: ByteBuffer): Unit

  @native def shardCreate(ctx: Long, comp: ByteBuffer, n: Long, fileOffset: Long, fileSize: Long): Long
  @native def shardDestroy(sh: Long): Unit
  /** sbh_shard_load: new resident bytes [fileOffset, fileOffset + n) of the same file, device buffers kept */
  @native def shardLoad(ctx: Long, sh: Long, comp: ByteBuffer, n: Long, fileOffset: Long): Unit
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
  /** sbh_split_records: one FileSplit of loadReadsAndPositions in one call; out = {blockStart, nBlocks,
    * flatSize, ownedFlat, firstFlat, firstVpos, nTrue, nRecords, nameBytes, cigarOps, bases, auxBytes} */
  @native def splitRecords(ctx: Long, sh: Long, start: Long, end: Long, blocksToCheck: Int, readsToCheck: Int,
                           maxReadSize: Int, decode: Boolean, out: Array[Long]): Unit
  /** out = {nRecords, nameBytes, cigarOps, bases, auxBytes} */
  @native def recordsScan(ctx: Long, sh: Long, first: Long, endFlat: Long, out: Array[Long]): Unit
  /** 18 (or 19, + vpos) direct buffers in sbh_records_out order, sized from recordsScan's `sizes` */
  @native def recordsFetch(ctx: Long, sh: Long, sizes: Array[Long], columns: Array[ByteBuffer]): Unit
  /** htsjdk-rewrite's BGZF writer (sbh_bgzf_compress_level; level 5 = htsjdk's bytes):
    * returns the file length written into `out` (capacity >= bgzfBound(n)). */
  @native def bgzfBound(n: Long): Long
  @native def bgzfCompress(ctx: Long, src: ByteBuffer, n: Long, level: Int, out: ByteBuffer): Long
  /** Blocks.apply's unindexed branch over a local file (mapped by the shim; sbh_find_blocks):
    * 4 longs per block {split index, start, compressedSize, uncompressedSize}. */
  @native def findBlocks(ctx: Long, path: String, starts: Array[Long], ends: Array[Long], blocksToCheck: Int,
                         window: Long): Array[Long]
  /** check-bam -s / full-check over the listed blocks of a local file of any size
    * (sbh_check_stream): out = {nWindows, positions, compBytes, nTrue, tp, fp, fn, unknown,
    * nSuccess, nClose, haloFinal}; null buffers skip their part. */
  @native def checkStream(ctx: Long, path: String, contigs: Array[Int], blocks: Array[Long], truthVpos: ByteBuffer,
                          nTruth: Long, full: Boolean, window: Long, halo: Long, readsToCheck: Int,
                          fpVpos: ByteBuffer, fnVpos: ByteBuffer, mismatchCap: Long, counts: ByteBuffer,
                          rbe: ByteBuffer, closeVpos: ByteBuffer, closeWord: ByteBuffer, closeCap: Long,
                          out: Array[Long]): Unit
  /** loadBamIntervals' record pass (sbh_records_scan_regions): out = {n, nameBytes, cigarOps,
    * bases, auxBytes} for recordsFetch. */
  @native def recordsScanRegions(ctx: Long, sh: Long, chunkBegin: Array[Long], chunkEnd: Array[Long],
                                 ivRef: Array[Int], ivBegin: Array[Long], ivEnd: Array[Long], out: Array[Long]): Unit
}

/** One executor GPU: one sbh_ctx, shared WITHOUT a lock by every task thread of the executor.  The
  * library allows any number of threads on one context as long as each shard is used by one thread
  * at a time (include/sparkbam.h, threading): every task below makes or reuses shards of its own
  * (GpuShard, GpuSplitWorker), each shard runs on its own HIP stream, and a failed call's detail is
  * kept per thread, so the shim's exception is always the calling task's.  This is the reference's
  * model, where each task builds its own channel and checker (CanLoadBam.scala:316-320,
  * PosChecker.scala:19-20).  (`lazy val` initialization is itself synchronized.) */
object Device {
  lazy val ctx: Long = Native.ctxCreate(sys.env.getOrElse("LOCAL_RANK", "0").toInt)
}

/** Compressed bytes [fileOffset, fileOffset + n) of a BGZF file, resident in HBM.  Used by one
  * thread at a time; `reload` moves it to other bytes of the same file, keeping its device buffers. */
class GpuShard(comp: ByteBuffer, private var n: Long, private var offset: Long, fileSize: Long, contigs: Array[Int])
  extends AutoCloseable {
  private val ctx = Device.ctx
  val sh: Long = Native.shardCreate(ctx, comp, n, offset, fileSize)
  Native.setContigs(ctx, sh, contigs)
  def fileOffset: Long = offset
  def atEof: Boolean = offset + n == fileSize
  private val nf = new Array[Long](2)
  def load(start: Long): Unit = Native.indexAndInflate(ctx, sh, start, nf)
  /** the resident bytes become [fileOffset, fileOffset + n) of the same file (sbh_shard_load) */
  def reload(comp: ByteBuffer, n: Long, fileOffset: Long): Unit = {
    Native.shardLoad(ctx, sh, comp, n, fileOffset)
    this.n = n
    this.offset = fileOffset
    nf(0) = 0
    nf(1) = 0
  }
  /** the block table a combined call (splitRecords) built: its size, for blocks() */
  def indexed(numBlocks: Long, flatSize: Long): Unit = { nf(0) = numBlocks; nf(1) = flatSize }
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
      // eager.Checker.nextReadStartWithDelta's None (eager/Checker.scala:134-162)
      case e: NativeException if e.status == Native.NO_READ_FOUND ⇒ None
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

/** Drop-in for bgzf/.../block/Stream.scala's SeekableStream (:79-121): a SUBCLASS of the reference's
  * own SeekableStream, so the reference's SeekableUncompressedBytes(blockStream) (UncompressedBytes
  * .scala:65-87) and every caller of it take it unchanged -- only where the stream is built changes
  * (GpuSeekableStream.uncompressedBytes, INTEGRATION.md).  Its blocks come from a WINDOW of the file
  * (compressed bytes [p, p + window) plus a halo, in one reused shard) indexed and inflated on the
  * device in one pass, the window's inflated bytes copied to the host once; the window replaces the
  * reference's 100-block LRU: a seek back into it (CanLoadBam.scala:349 seeks to the split's first
  * record right after FindRecordStart read past it) re-inflates nothing.  seek(newPos) is the
  * reference's own (clear and reposition unless already there); _advance reads the block at the
  * channel's position, and the empty block that ends the stream answers None (Stream.scala:56-58).
  * Mirrored by spark_bam_amd.seekable.SeekableStream (tests/test_seekable_gpu.py). */
class GpuSeekableStream(ch: SeekableByteChannel, window: Long = 16L << 20, halo: Long = 1L << 20)
  extends SeekableStream(ch) {

  private var buf: ByteBuffer = _
  private var shard: GpuShard = _
  private var contigs: Array[Int] = Array.empty
  private var starts: Array[Long] = Array.empty  // the window's blocks (sorted starts) and their
  private var table: Array[Long] = Array.empty   // (start, ustart, csize, hsize, usize, flags) rows
  private var flat: Array[Byte] = Array.empty    // the window's inflated bytes, host copy
  private var wHi = -1L
  var windowsLoaded = 0

  /** index + inflate the blocks from the block start p over [p, p + w + halo) */
  private[gpu] def load(p: Long, w: Long = window): Unit = {
    val size = ch.size
    val m = math.min(size - p, w + halo)
    if (buf == null || buf.capacity < m) {
      if (buf != null) Native.hostFree(buf)
      buf = Native.hostAlloc(math.max(m, 1L << 20))
    }
    buf.clear()
    buf.limit(m.toInt)
    val back = ch.position()
    ch.seek(p)
    ch.readFully(buf)
    ch.seek(back)
    buf.flip()
    if (shard == null) shard = new GpuShard(buf, m, p, size, contigs)
    else shard.reload(buf, m, p)
    shard.load(p)
    table = shard.blocks(0, shard.numBlocks)
    starts = Array.tabulate(shard.numBlocks.toInt)(i ⇒ table(6 * i))
    flat = if (shard.flatSize > 0) shard.flat(0, shard.flatSize.toInt) else Array.empty
    wHi = p + m
    windowsLoaded += 1
  }

  private def row(p: Long): Int = {
    val i = java.util.Arrays.binarySearch(starts, p)
    if (i < 0 || (table(6 * i + 5) & 2) != 0) -1 else i  // (2: a block cut off by the window's end)
  }

  override protected def _advance: Option[Block] = {
    val start = compressedBytes.position()
    if (start >= compressedBytes.size) return None  // (the reference's EOFException -> None)
    var i = row(start)
    if (i < 0) { load(start); i = row(start) }
    val (ustart, csize, usize, flags) = (table(6 * i + 1), table(6 * i + 2), table(6 * i + 4), table(6 * i + 5))
    compressedBytes.seek(start + csize)
    if ((flags & 1) != 0) None  // dataLength == 2: the empty block ending the stream
    else Some(Block(java.util.Arrays.copyOfRange(flat, ustart.toInt, (ustart + usize).toInt), start, csize.toInt))
  }

  /** FindRecordStart.withDelta from Pos(start, 0) on the window's shard (grown x4 while the search
    * needs bytes past it): Some((pos, positions skipped)) or None. */
  def findRecordStart(start: Long, contigLengths: Array[Int], readsToCheck: Int,
                      maxReadSize: Int): Option[(Pos, Int)] = {
    if (!java.util.Arrays.equals(contigs, contigLengths)) {
      contigs = contigLengths
      if (shard != null) Native.setContigs(Device.ctx, shard.sh, contigs)
    }
    var w = window
    if (shard == null || row(start) < 0) load(start, w)
    while (true) {
      try {
        return shard.findRecordStart(table(6 * row(start) + 1), readsToCheck, maxReadSize).map {
          case (f, d) ⇒ (shard.posOf(f), d)
        }
      } catch {
        case e: NeedHaloException if wHi < ch.size ⇒ w *= 4; load(start, w)
      }
    }
    None
  }

  override def close(): Unit = {
    if (shard != null) { shard.close(); shard = null }
    if (buf != null) { Native.hostFree(buf); buf = null }
    super.close()
  }
}

object GpuSeekableStream {
  /** the reference's SeekableUncompressedBytes over a GPU-inflated SeekableStream: what
    * SeekableUncompressedBytes(ch) (UncompressedBytes.scala:79-86) builds, with the GPU stream */
  def uncompressedBytes(ch: SeekableByteChannel, window: Long = 16L << 20): SeekableUncompressedBytes =
    SeekableUncompressedBytes(new GpuSeekableStream(ch, window))
}

/** Drop-in for check/.../spark/FindRecordStart.scala:11-71 on the GPU: the first eager-true
  * position at/after Pos(start, 0) within maxReadSize positions.  Same signature.  When the
  * caller's `uncompressedBytes` is GPU-backed (GpuSeekableStream) the search runs on that view's
  * window shard -- the blocks its next reads will come from -- and the view is left at the found
  * record, as the reference's withDelta leaves it (FindRecordStart.scala:30-63); otherwise a shard of
  * the file from `start` (grown x4 while the search needs bytes past it). */
object GpuFindRecordStart {
  def apply(path: Path,
            start: Long)(
      implicit
      uncompressedBytes: SeekableUncompressedBytes,
      contigLengths: ContigLengths,
      readsToCheck: ReadsToCheck,
      maxReadSize: MaxReadSize): Pos = {
    val found = uncompressedBytes.blockStream match {
      case g: GpuSeekableStream ⇒
        g.findRecordStart(start, GpuShard.contigArray(contigLengths), readsToCheck.n, maxReadSize.n).map(_._1)
      case _ ⇒
        withDelta(path, Pos(start, 0)).map(_._1)
    }
    found match {
      case Some(pos) ⇒
        uncompressedBytes.seek(pos)
        pos
      case None ⇒ throw NoReadFoundException(path, start, maxReadSize)
    }
  }

  /** FindRecordStart.withDelta: Some((pos, positions skipped)) or None */
  def withDelta(path: Path, start: Pos, halo0: Long = 1L << 20)(
      implicit
      contigLengths: ContigLengths,
      readsToCheck: ReadsToCheck,
      maxReadSize: MaxReadSize): Option[(Pos, Int)] = {
    val ch = SeekableByteChannel(path)
    try {
      var halo = halo0
      while (true) {
        val s = GpuShard.read(ch, start.blockPos, halo, GpuShard.contigArray(contigLengths))
        try {
          s.load(start.blockPos)
          return s.findRecordStart(s.flatOf(start), readsToCheck.n, maxReadSize.n).map {
            case (f, delta) ⇒ (s.posOf(f), delta)
          }
        } catch {
          case e: NeedHaloException ⇒
            if (start.blockPos + halo >= ch.size) throw e
            halo *= 4
        } finally s.close()
      }
      None
    } finally ch.close()
  }
}

/** RecordStream over the records a shard's device pass found (RecordStream.scala:16-41):
  * (Pos, SAMRecord) in file order.  The record starts come from the GPU (sbh_records_scan /
  * sbh_records_scan_regions left them, "flat" column); the records' bytes are read out of HBM in
  * one copy and each SAMRecord is built exactly as htsjdk's BAMRecordCodec.decode builds it
  * (the 32 fixed-field bytes after block_size, then SAMRecordFactory.createBAMRecord over the
  * variable-length rest), so the objects equal the reference's.  `sizes` are the scan's
  * {n, nameBytes, cigarOps, bases, auxBytes}.  Everything is copied out on construction: the
  * shard may be closed right after. */
class GpuRecordIterator(shard: GpuShard, sizes: Array[Long], header: SAMFileHeader)
  extends Iterator[(Pos, SAMRecord)] {
  private val n = sizes(0).toInt
  // the starts (flat) and their canonical Pos as htsjdk virtual positions, both computed on the
  // device (sbh_records_out fields 0 and 18: a start at a block's end is Pos(next, 0))
  private val (flats, vposs): (Array[Long], Array[Long]) = {
    val b = ByteBuffer.allocateDirect(math.max(8, 8 * n)).order(ByteOrder.LITTLE_ENDIAN)
    val v = ByteBuffer.allocateDirect(math.max(8, 8 * n)).order(ByteOrder.LITTLE_ENDIAN)
    val cols = new Array[ByteBuffer](19)
    cols(0) = b
    cols(18) = v
    Native.recordsFetch(Device.ctx, shard.sh, sizes, cols)
    (Array.tabulate(n)(i ⇒ b.getLong(8 * i)), Array.tabulate(n)(i ⇒ v.getLong(8 * i)))
  }
  // the bytes of [first record, end of the last record), read once
  private val (lo, raw) =
    if (n == 0) (0L, ByteBuffer.allocate(0))
    else {
      val last = flats(n - 1)
      val len4 = ByteBuffer.wrap(shard.flat(last, 4)).order(ByteOrder.LITTLE_ENDIAN).getInt(0)
      val hi = last + 4 + (len4.toLong & 0xffffffffL)
      val b = ByteBuffer.allocateDirect((hi - flats(0)).toInt).order(ByteOrder.LITTLE_ENDIAN)
      Native.readFlat(Device.ctx, shard.sh, flats(0), hi - flats(0), b)
      (flats(0), b)
    }
  private val factory = DefaultSAMRecordFactory.getInstance
  private var i = 0

  override def hasNext: Boolean = i < n

  override def next(): (Pos, SAMRecord) = {
    val f = flats(i)
    i += 1
    val o = (f - lo).toInt
    val blockSize = raw.getInt(o)
    val binMqNl = raw.getInt(o + 12)
    val flagNc = raw.getInt(o + 16)
    val rest = new Array[Byte](blockSize - 32)
    val dup = raw.duplicate()
    dup.position(o + 36)
    dup.get(rest)
    val rec = factory.createBAMRecord(
      header,
      raw.getInt(o + 4),                // referenceID
      raw.getInt(o + 8) + 1,            // coordinate (1-based)
      (binMqNl & 0xff).toShort,         // readNameLength
      ((binMqNl >>> 8) & 0xff).toShort, // mappingQuality
      binMqNl >>> 16,                   // indexingBin
      flagNc & 0xffff,                  // cigarLen
      flagNc >>> 16,                    // flags
      raw.getInt(o + 20),               // readLen
      raw.getInt(o + 24),               // mateReferenceID
      raw.getInt(o + 28) + 1,           // mateCoordinate
      raw.getInt(o + 32),               // insertSize
      rest)
    Pos(vposs(i - 1)) → rec
  }
}

/** One executor task thread's reusable device state for GpuSplitPartition: a page-locked buffer the
  * split's bytes are read into and ONE shard whose device buffers (compressed bytes, tokens, flat
  * bytes, bitmap, block table, record starts) serve every split the thread runs (sbh_shard_load,
  * grow-only), so a split costs no host or device allocation.  Per thread (ThreadLocal): Spark runs
  * an executor's tasks on a pool of threads, and a shard is one thread's at a time.  Mirrored by
  * spark_bam_amd.canloadbam.SplitWorker. */
class GpuSplitWorker(val contigs: Array[Int]) extends AutoCloseable {
  private var buf: ByteBuffer = _
  private var shard: GpuShard = _
  private var fileSize = -1L

  /** the thread's shard holding [lo, min(size, lo + n)) of the channel's file */
  def load(ch: SeekableByteChannel, lo: Long, n: Long): GpuShard = {
    val size = ch.size
    val m = math.min(size - lo, n)
    if (buf == null || buf.capacity < m) {
      if (buf != null) Native.hostFree(buf)
      buf = Native.hostAlloc(math.max(m + (m >> 3), 1L << 20))  // (room for a grown halo)
    }
    buf.clear()
    buf.limit(m.toInt)
    ch.seek(lo)
    ch.readFully(buf)
    buf.flip()
    if (shard == null || fileSize != size) {
      if (shard != null) shard.close()
      shard = new GpuShard(buf, m, lo, size, contigs)
      fileSize = size
    } else shard.reload(buf, m, lo)
    shard
  }

  override def close(): Unit = {
    if (shard != null) { shard.close(); shard = null }
    if (buf != null) { Native.hostFree(buf); buf = null }
  }
}

object GpuSplitWorker {
  private val local = new ThreadLocal[GpuSplitWorker]
  /** the calling thread's worker; the contig lengths are set on its shard, so another file's
    * contigs replace it */
  def get(contigs: Array[Int]): GpuSplitWorker = {
    val w = local.get
    if (w != null && java.util.Arrays.equals(w.contigs, contigs)) w
    else {
      if (w != null) w.close()
      val n = new GpuSplitWorker(contigs)
      local.set(n)
      n
    }
  }
}

/** loadReadsAndPositions' per-split body (CanLoadBam.scala:316-356) on the executor's GPU: the
  * split's compressed bytes [start, end) plus a halo in the task thread's reused shard, then ONE
  * library call (sbh_split_records): FindBlockStart(start), index + inflate from it, the eager check
  * over the owned positions [0, flat(Pos(end, 0))), FindRecordStart from Pos(blockStart, 0), and
  * the record starts while pos < Pos(end, 0) (RecordStream.takeWhile).  The halo grows x4 while an
  * answer -- the split's last record included -- needs bytes past it.  Mirrored call for call by
  * spark_bam_amd.canloadbam.SplitWorker.split (tests/test_canloadbam_gpu.py, tests/test_threads_gpu.py). */
object GpuSplitPartition {
  def apply(path: Path, start: Long, end: Long, header: SAMFileHeader, contigs: Array[Int],
            bgzfBlocksToCheck: Int, readsToCheck: Int, maxReadSize: Int,
            halo0: Long = 1L << 20): Iterator[(Pos, SAMRecord)] = {
    val ch = SeekableByteChannel(path)
    val w = GpuSplitWorker.get(contigs)
    try {
      var halo = halo0
      while (true) {
        val s = w.load(ch, start, end - start + halo)
        try {
          val out = new Array[Long](12)
          try Native.splitRecords(Device.ctx, s.sh, start, end, bgzfBlocksToCheck, readsToCheck, maxReadSize,
                                  false, out)
          catch Native.rethrow(path)
          s.indexed(out(1), out(2))
          // (the iterator copies the starts and the records' bytes out: the shard is free again)
          return new GpuRecordIterator(s, out.slice(7, 12), header)
        } catch {
          case e: NeedHaloException if end + halo < ch.size ⇒ halo *= 4
          // a record (or the chain's next one) past the resident bytes: more halo, as the reference
          // would simply read on
          case e: NativeException
            if (e.status == Native.NOT_FOUND || e.status == Native.BAD_RECORD) && end + halo < ch.size ⇒
            halo *= 4
        }
      }
      Iterator.empty
    } finally ch.close()
  }
}

/** loadBamIntervals' per-partition body (CanLoadBam.scala:120-154) on the executor's GPU: the
  * partition's chunks whose block ranges lie within `mergeGap` of each other share one shard
  * [first chunk's block, last chunk's end block + halo); index + inflate, the eager check over
  * the chunks' flat span, then sbh_records_scan_regions keeps the records starting in a chunk
  * whose region meets the intervals (region(record) as in CanLoadBam.scala:447-454).  Mirrored
  * by spark_bam_amd.canloadbam.intervals_partition. */
object GpuIntervalsPartition {
  def apply(path: Path, chunks: Seq[Chunk], ivRef: Array[Int], ivBegin: Array[Long], ivEnd: Array[Long],
            header: SAMFileHeader, contigs: Array[Int], readsToCheck: Int,
            halo0: Long = 1L << 18, mergeGap: Long = 1L << 20): Iterator[SAMRecord] = {
    val groups = scala.collection.mutable.ArrayBuffer[(Long, Long, Seq[Chunk])]()
    for (c ← chunks) {
      val (lo, hi) = (c.start.blockPos, c.end.blockPos)
      if (groups.nonEmpty && lo <= groups.last._2 + mergeGap) {
        val g = groups.last
        groups(groups.size - 1) = (g._1, math.max(g._2, hi), g._3 :+ c)
      } else groups += ((lo, hi, Seq(c)))
    }
    val ch = SeekableByteChannel(path)
    try {
      groups.iterator.flatMap {
        case (lo, hi, cs) ⇒
          var halo = halo0
          var out: Vector[SAMRecord] = null
          while (out == null) {
            val s = GpuShard.read(ch, lo, hi - lo + halo, contigs)
            try {
              s.load(lo)
              def flat(p: Pos): Long = if (p.blockPos >= ch.size) s.flatSize else s.flatOf(p)
              val fb = cs.map(c ⇒ flat(c.start)).toArray
              val fe = cs.map(c ⇒ math.min(flat(c.end), s.flatSize)).toArray
              if (fe.max > fb.min) Native.checkEager(Device.ctx, s.sh, fb.min, fe.max, readsToCheck, null)
              val sizes = new Array[Long](5)
              Native.recordsScanRegions(Device.ctx, s.sh, fb, fe, ivRef, ivBegin, ivEnd, sizes)
              out = new GpuRecordIterator(s, sizes, header).map(_._2).toVector
            } catch {
              // an eager check reading on, a chunk end or a kept record past the shard: grow it
              case e: NeedHaloException if hi + halo < ch.size ⇒ halo *= 4
              case e: NativeException
                if (e.status == Native.NOT_FOUND || e.status == Native.BAD_RECORD) && hi + halo < ch.size ⇒
                halo *= 4
            } finally s.close()
          }
          out
      }.toVector.iterator
    } finally ch.close()
  }
}

/** CanLoadBam with the hot path on the GPU: the same five entry points with the reference's
  * parameter lists (load/.../CanLoadBam.scala:61-405); Spark partitioning is the reference's
  * (one task per Hadoop FileSplit through SplitRDD(FileSplits.asJava(path, splitSize)); one per
  * cappedCostGroups chunk group for intervals), and each task's FindBlockStart / inflate /
  * FindRecordStart / record boundaries run on its executor's GPU (GpuSplitPartition,
  * GpuIntervalsPartition).  Records are htsjdk SAMRecords built from the records' bytes exactly as
  * BAMRecordCodec builds them.  `import spark_bam_gpu._` in place of `import spark_bam._`
  * (jni/spark_bam_gpu.scala) puts these methods on SparkContext. */
trait GpuCanLoadBam extends CanLoadBam {

  override def loadBam(path: Path,
                       splitSize: MaxSplitSize = MaxSplitSize(),
                       bgzfBlocksToCheck: BGZFBlocksToCheck = default[BGZFBlocksToCheck],
                       readsToCheck: ReadsToCheck = default[ReadsToCheck],
                       maxReadSize: MaxReadSize = default[MaxReadSize]
                      ): RDD[SAMRecord] =
    loadReadsAndPositions(path, splitSize, bgzfBlocksToCheck, readsToCheck, maxReadSize).values

  override def loadSplitsAndReads(path: Path,
                                  splitSize: MaxSplitSize = MaxSplitSize(),
                                  bgzfBlocksToCheck: BGZFBlocksToCheck = default[BGZFBlocksToCheck],
                                  readsToCheck: ReadsToCheck = default[ReadsToCheck],
                                  maxReadSize: MaxReadSize = default[MaxReadSize]
                                 ): BAMRecordRDD = {
    val positionsAndReadsRDD = loadReadsAndPositions(path, splitSize, bgzfBlocksToCheck, readsToCheck, maxReadSize)
    val endPos = Pos(path.size, 0)
    // the first record of every non-empty partition, sliding2 with Pos(fileSize, 0) (:283-297)
    val splits =
      positionsAndReadsRDD
        .mapPartitions(it ⇒ if (it.hasNext) Iterator(it.next._1) else Iterator())
        .collect
        .sliding2(endPos)
        .map(Split(_))
        .toVector
    BAMRecordRDD(splits, positionsAndReadsRDD.values)
  }

  override def loadReadsAndPositions(path: Path,
                                     splitSize: MaxSplitSize,
                                     bgzfBlocksToCheck: BGZFBlocksToCheck,
                                     readsToCheck: ReadsToCheck,
                                     maxReadSize: MaxReadSize
                                    ): RDD[(Pos, SAMRecord)] = {
    val headerBroadcast = sc.broadcast(Header(path))
    val contigs = GpuShard.contigArray(ContigLengths(path))
    val (k, r, m) = (bgzfBlocksToCheck.n, readsToCheck.n, maxReadSize.n)
    SplitRDD(FileSplits.asJava(path, splitSize))
      .flatMap {
        case (start, end) ⇒
          GpuSplitPartition(path, start, end, headerBroadcast.value, contigs, k, r, m)
      }
  }

  override def loadReads(path: Path,
                         bgzfBlocksToCheck: BGZFBlocksToCheck = default[BGZFBlocksToCheck],
                         readsToCheck: ReadsToCheck = default[ReadsToCheck],
                         maxReadSize: MaxReadSize = default[MaxReadSize],
                         splitSize: MaxSplitSize = MaxSplitSize()): RDD[SAMRecord] =
    path.extension match {
      case "bam" ⇒ loadBam(path, splitSize, bgzfBlocksToCheck, readsToCheck, maxReadSize)
      case _ ⇒ super.loadReads(path, bgzfBlocksToCheck, readsToCheck, maxReadSize, splitSize)  // sam / cram
    }

  override def loadBamIntervals(path: Path,
                                intervals: LociSet,
                                splitSize: MaxSplitSize,
                                estimatedCompressionRatio: EstimatedCompressionRatio): RDD[SAMRecord] = {
    if (path.toString.endsWith(".sam"))
      return super.loadBamIntervals(path, intervals, splitSize, estimatedCompressionRatio)
    val header = Header(path)
    val headerBroadcast = sc.broadcast(header)
    val contigs = GpuShard.contigArray(header.contigLengths)
    // the merged intervals, 0-based half-open, as (contig index, begin, end): the same
    // htsjdk intervals getIntevalChunks queries the BAI with (CanLoadBam.scala:425-436)
    val samHeader: SAMFileHeader = header
    val dict = samHeader.getSequenceDictionary
    val ivs = intervals.toHtsJDKIntervals.toArray
      .map(i ⇒ (dict.getSequenceIndex(i.getContig), i.getStart - 1L, i.getEnd.toLong))
      .sorted
    val (ivRef, ivBegin, ivEnd) = (ivs.map(_._1), ivs.map(_._2), ivs.map(_._3))
    val chunks = CanLoadBam.getIntevalChunks(path, intervals)
    val chunkPartitions =
      chunks
        .cappedCostGroups(_.size(estimatedCompressionRatio), splitSize.toDouble)
        .map(_.toVector)
        .toVector
    sc
      .parallelize(chunkPartitions, math.max(1, chunkPartitions.size))
      .mapPartitions {
        groups ⇒
          val h: SAMFileHeader = headerBroadcast.value
          groups.flatMap(cs ⇒ GpuIntervalsPartition(path, cs, ivRef, ivBegin, ivEnd, h, contigs, 10))
      }
  }
}

/** Blocks.apply's unindexed branch (check/.../check/Blocks.scala:141-206) for a local file:
  * FindBlockStart per split, then MetadataStream to the split's end, on the device
  * (sbh_find_blocks); per split the Metadata(start, compressedSize, uncompressedSize) list. */
object GpuBlocks {
  def unindexed(path: Path, splits: Seq[(Long, Long)], bgzfBlocksToCheck: Int = 5,
                window: Long = 1L << 30): Vector[Vector[Metadata]] = {
    val v =
      try Native.findBlocks(Device.ctx, path.toString, splits.map(_._1).toArray, splits.map(_._2).toArray,
                            bgzfBlocksToCheck, window)
      catch Native.rethrow(path)
    val per = Array.fill(splits.size)(Vector.newBuilder[Metadata])
    for (i ← 0 until v.length / 4)
      per(v(4 * i).toInt) += Metadata(v(4 * i + 1), v(4 * i + 2).toInt, v(4 * i + 3).toInt)
    per.map(_.result()).toVector
  }
}

/** check-bam -s (CheckerApp.scala:65-227 + CallPartition.scala:23-54) and full-check
  * (FullCheck.scala:65-86,142-192) over Blocks.apply's blocks of a local file of any size, the
  * file streamed through HBM (sbh_check_stream): the totals the apps print, the mismatching
  * positions (first mismatchCap), and with full the Counts / readsBeforeError histograms by
  * numNonZeroFields and the close calls.  Mirrored by spark_bam_amd.api.check_bam / full_check. */
object GpuCheckStream {
  case class Totals(windows: Long, positions: Long, compressedBytes: Long, trueCalls: Long, tp: Long, fp: Long,
                    fn: Long, unknown: Long, successes: Long, closeCalls: Long)

  case class Calls(totals: Totals, falsePositives: Seq[Pos], falseNegatives: Seq[Pos], counts: Array[Long],
                   readsBeforeError: Array[Long], close: Seq[(Pos, Int)])

  def apply(path: Path, contigLengths: ContigLengths, blocks: Array[Long], records: Option[Array[Long]],
            full: Boolean, readsToCheck: Int = 10, window: Long = 1L << 30, halo: Long = 4L << 20,
            mismatchCap: Int = 1 << 20, closeCap: Int = 1 << 22): Calls = {
    def longs(n: Int) = ByteBuffer.allocateDirect(8 * math.max(1, n)).order(ByteOrder.LITTLE_ENDIAN)
    val truth = records.map { r ⇒ val b = longs(r.length); b.asLongBuffer.put(r); b }
    val (fp, fn) = if (records.isDefined) (longs(mismatchCap), longs(mismatchCap)) else (null, null)
    val (counts, rbe) = if (full) (longs(21 * 19), longs(21 * 64)) else (null, null)
    val (cv, cw) =
      if (full) (longs(closeCap), ByteBuffer.allocateDirect(4 * closeCap).order(ByteOrder.LITTLE_ENDIAN))
      else (null, null)
    val out = new Array[Long](11)
    Native.checkStream(Device.ctx, path.toString, GpuShard.contigArray(contigLengths), blocks, truth.orNull,
                       records.map(_.length.toLong).getOrElse(0L), full, window, halo, readsToCheck, fp, fn,
                       mismatchCap, counts, rbe, cv, cw, closeCap, out)
    val t = Totals(out(0), out(1), out(2), out(3), out(4), out(5), out(6), out(7), out(8), out(9))
    def poss(b: ByteBuffer, n: Long) =
      if (b == null) Seq() else (0 until math.min(n, mismatchCap.toLong).toInt).map(i ⇒ Pos(b.getLong(8 * i)))
    def arr(b: ByteBuffer, n: Int) = if (b == null) Array.empty[Long] else Array.tabulate(n)(i ⇒ b.getLong(8 * i))
    val close =
      if (!full) Seq()
      else (0 until math.min(t.closeCalls, closeCap.toLong).toInt).map(i ⇒ (Pos(cv.getLong(8 * i)), cw.getInt(4 * i)))
    Calls(t, poss(fp, t.fp), poss(fn, t.fn), arr(counts, 21 * 19), arr(rbe, 21 * 64), close)
  }
}
