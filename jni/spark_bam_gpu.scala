// spark_bam_gpu.scala -- the GPU twin of load/src/main/scala/spark_bam/package.scala:5-13:
// `import spark_bam_gpu._` in place of `import spark_bam._` gives SparkContext (and
// hammerlab's spark Context) the CanLoadBam methods with the hot path on the executors' GPUs
// (org.hammerlab.bam.gpu.GpuCanLoadBam, jni/Native.scala).
import org.apache.spark.SparkContext
import org.hammerlab.bam.gpu.GpuCanLoadBam
import org.hammerlab.spark.Context

package object spark_bam_gpu {
  implicit class GpuLoadBamSparkContext(val sc: SparkContext)
    extends GpuCanLoadBam

  implicit class GpuLoadBamContext(val ctx: Context)
    extends GpuCanLoadBam {
    override implicit def sc: SparkContext = ctx
  }
}
