// GpuRound.scala — Scala side of the MI355X plugin for the reference (PSync).
//
// Drop into the reference build as src/main/scala/psync/gpu/GpuRound.scala and
// put libpsg_jni.so (integration/jni/psg_jni.c) + libpsg.so on java.library.path.
// Not compiled in this repository's CI (no JVM in the image).
//
// It replaces, for simulation, `alg.startInstance(id, io)` on a netty Runtime
// (psync/Algorithm.scala:36-42, psync/runtime/Runtime.scala:167-177) by a batched
// lockstep HO execution of [begin, begin+count) instances on one GPU, or split
// over several (GpuConfig.devices: one host thread per device inside the library,
// the per-instance executor pool of psync/runtime/Runtime.scala:43-57, 126-128),
// with the algorithm's Spec checked after every round.
package psync.gpu

import psync.Algorithm

/** JNI entry points (one per psg.h function). */
object GpuRoundNative {
  System.loadLibrary("psg_jni")
  @native def create(alg: Int, n: Int, rounds: Int, seed: Long, valueRange: Int, param: Int, param2: Int,
                     realParam: Double, tiebreak: Int, device: Int, variant: Int, batchCapacity: Long, dropLog2: Int,
                     goodP32: Int, goodMin: Int, crashFmax: Int, hoMin: Int, selfBit: Boolean,
                     devices: Array[Int]): Long
  @native def loadInputs(ctx: Long, begin: Long, count: Long, init: Array[Int]): Unit
  @native def loadInputsF64(ctx: Long, begin: Long, count: Long, init: Array[Double]): Unit
  @native def copyDecisionsF64(ctx: Long, decision: Array[Double], decisionRound: Array[Int]): Unit
  @native def runBatch(ctx: Long, begin: Long, count: Long, perInstance: Array[Byte]): Array[Long]
  @native def runBatchSpec(ctx: Long, begin: Long, count: Long, code: Array[Int], slotEntry: Array[Int],
                           slotFlags: Array[Int], termEntry: Int, nVars: Int, alg: Int, modulePath: String,
                           perInstance: Array[Byte]): Array[Long]
  @native def copyDecisions(ctx: Long, decision: Array[Int], decisionRound: Array[Int]): Unit
  @native def compileSpec(text: String, alg: Int): Array[Int]
  @native def compileSpecNames(text: String, alg: Int): String
  @native def compileSpecNative(text: String, alg: Int, fused: Boolean, n: Int): String
  @native def fetch(ctx: Long, ids: Array[Long], sums: Array[Byte], records: Array[Int]): Unit
  @native def loadSchedule(ctx: Long, begin: Long, count: Long, ho: Array[Long], crash: Array[Int]): Unit
  @native def clearSchedule(ctx: Long): Unit
  @native def materializeSchedule(ctx: Long, begin: Long, count: Long, ho: Array[Long], crash: Array[Int]): Unit
  @native def destroy(ctx: Long): Unit
}

/** HO schedule (faults are HO sets, psync/Process.scala:14). */
case class HOSchedule(dropLog2: Int = 3, goodRound: Double = 0.25, goodMin: Int = -1,
                      crashFmax: Int = -1, hoMin: Int = -1, selfBit: Boolean = true)

/** param: OTR/OTR2 afterDecision, FloodMin f, KSet k, KSetEarlyStopping t, EpsilonConsensus f;
  * param2: KSetEarlyStopping k; realParam: EpsilonConsensus epsilon. */
case class GpuConfig(n: Int, rounds: Int, seed: Long = 1L, valueRange: Int = 4, param: Int = 0,
                     schedule: HOSchedule = HOSchedule(), tiebreakChamp: Boolean = true,
                     device: Int = 0, batchCapacity: Long = 1L << 20, variant: Int = 0,
                     param2: Int = 0, realParam: Double = 0.0, devices: Seq[Int] = Nil) {
  require(n >= 1 && n <= 256, "n out of range 1..256")
  require(rounds >= 1 && rounds <= 250, "rounds out of range 1..250")
  require(devices.length <= 16, "at most 16 devices per context")
}

/** Node-level result of a batch (psg_summary). processRounds counts every instance's n * R
  * process-rounds (SURVEY §8d); activeProcessRounds those in which the process took a step;
  * liveInstanceRounds the instance-rounds in which some process was still active. */
case class GpuResult(instances: Long, processRounds: Long, activeProcessRounds: Long, liveInstanceRounds: Long,
                     failCount: Array[Long], decidedProcesses: Long, digest: Long, termHist: Array[Long],
                     kernelNs: Long)

object GpuRound {
  /** Algorithm ids keyed on the reference class (SURVEY §8b). */
  val registry: Map[String, Int] = Map(
    "example.OTR" -> 1, "example.LastVoting" -> 2, "example.FloodMin" -> 3,
    "example.KSetAgreement" -> 4, "example.BenOr" -> 5, "example.OTR2" -> 6,
    "example.ShortLastVoting" -> 7, "example.KSetEarlyStopping" -> 8, "example.EpsilonConsensus" -> 9)
  private val realValued = Set(9)

  def algId(alg: Algorithm[_, _]): Int =
    registry.getOrElse(alg.getClass.getName,
      throw new IllegalArgumentException("no GPU kernel for " + alg.getClass.getName))

  /** psg_summary as the long[] the shim returns (struct order, include/psg.h ABI 4). */
  private def summary(a: Array[Long], rounds: Int): GpuResult = {
    val nChecks = 12
    val h = 6 + nChecks  // term_hist offset
    GpuResult(a(0), a(1), a(2), a(3), a.slice(4, 4 + nChecks), a(4 + nChecks), a(5 + nChecks),
              a.slice(h, h + rounds + 2), a(a.length - 1))
  }

  /** Run instances [begin, begin+count) of `alg` in lockstep on one GPU. `init`
    * (optional, count*n) plays ConsensusIO.initialValue; `decide` receives the
    * ConsensusIO.decide callbacks (instance, pid, value, round) afterwards. */
  private def create(id: Int, cfg: GpuConfig): Long = {
    val s = cfg.schedule
    GpuRoundNative.create(id, cfg.n, cfg.rounds, cfg.seed, cfg.valueRange, cfg.param, cfg.param2, cfg.realParam,
      if (cfg.tiebreakChamp) 0 else 1, cfg.device, cfg.variant, cfg.batchCapacity, s.dropLog2,
      math.min(s.goodRound * 4294967296.0, 4294967295.0).toLong.toInt, s.goodMin, s.crashFmax, s.hoMin, s.selfBit,
      if (cfg.devices.isEmpty) null else cfg.devices.toArray)
  }

  private def checkRange(cfg: GpuConfig, begin: Long, count: Long): Unit = {
    require(begin >= 0 && count >= 0, "begin / count must be >= 0")
    require(count <= cfg.batchCapacity, s"count $count exceeds batchCapacity ${cfg.batchCapacity}")
  }

  /** RealConsensusIO algorithms (EpsilonConsensus, example/Epsilon.scala:10-13): Double
    * initial values and decide callbacks. */
  def runReal(alg: Algorithm[_, _], cfg: GpuConfig, begin: Long, count: Long, init: Option[Array[Double]] = None,
              decide: Option[(Long, Int, Double, Int) => Unit] = None): GpuResult = {
    val id = algId(alg)
    if (!realValued(id)) throw new IllegalArgumentException(alg.getClass.getName + " is not real-valued")
    checkRange(cfg, begin, count)
    init.foreach(a => require(a.length == count * cfg.n, s"init must hold count * n = ${count * cfg.n} values"))
    val ctx = create(id, cfg)
    try {
      GpuRoundNative.loadInputsF64(ctx, begin, count, init.orNull)
      val res = summary(GpuRoundNative.runBatch(ctx, begin, count, null), cfg.rounds)
      decide.foreach { cb =>
        val cells = (count * cfg.n).toInt
        val d = new Array[Double](cells)
        val r = new Array[Int](cells)
        GpuRoundNative.copyDecisionsF64(ctx, d, r)
        var i = 0
        while (i < cells) {
          if (r(i) >= 0) cb(begin + i / cfg.n, i % cfg.n, d(i), r(i))
          i += 1
        }
      }
      res
    } finally GpuRoundNative.destroy(ctx)
  }

  /** The seeded HO sets of instances [begin, begin+count) as data: ho(((i*R + k)*n + p)*W + w) = word w
    * of HO(p) in round k (bit q: p hears q), crash(i*n + p) = crash round or -1. */
  def materialize(alg: Algorithm[_, _], cfg: GpuConfig, begin: Long, count: Long): (Array[Long], Array[Int]) = {
    val W = (cfg.n + 63) / 64
    val ho = new Array[Long]((count * cfg.rounds * cfg.n * W).toInt)
    val crash = new Array[Int]((count * cfg.n).toInt)
    val ctx = create(algId(alg), cfg.copy(batchCapacity = math.max(1L, count)))
    try GpuRoundNative.materializeSchedule(ctx, begin, count, ho, crash)
    finally GpuRoundNative.destroy(ctx)
    (ho, crash)
  }

  /** Run instances under explicit HO sets (psg_load_schedule): a counterexample file's schedule,
    * or any schedule built in the JVM. */
  def runExplicit(alg: Algorithm[_, _], cfg: GpuConfig, begin: Long, count: Long, ho: Array[Long],
                  crash: Option[Array[Int]] = None, init: Option[Array[Int]] = None): GpuResult = {
    checkRange(cfg, begin, count)
    val W = (cfg.n + 63) / 64
    require(ho.length == count * cfg.rounds * cfg.n * W, s"ho must hold count * R * n * W = ${count * cfg.rounds * cfg.n * W} words")
    crash.foreach(a => require(a.length == count * cfg.n, s"crash must hold count * n = ${count * cfg.n} rounds"))
    init.foreach(a => require(a.length == count * cfg.n, s"init must hold count * n = ${count * cfg.n} values"))
    val ctx = create(algId(alg), cfg)
    try {
      GpuRoundNative.loadInputs(ctx, begin, count, init.orNull)
      GpuRoundNative.loadSchedule(ctx, begin, count, ho, crash.orNull)
      summary(GpuRoundNative.runBatch(ctx, begin, count, null), cfg.rounds)
    } finally GpuRoundNative.destroy(ctx)
  }

  /** Per-process (decision, decisionRound, haltRound, finalX), 4 ints each, of instances
    * [begin, begin+count) (psg_fetch_instances) with the given initial values (else seeded). */
  def records(alg: Algorithm[_, _], cfg: GpuConfig, begin: Long, count: Int,
              init: Option[Array[Int]] = None): Array[Int] = {
    require(begin >= 0 && count >= 0, "begin / count must be >= 0")
    init.foreach(a => require(a.length == count.toLong * cfg.n, s"init must hold count * n = ${count.toLong * cfg.n} values"))
    val ctx = create(algId(alg), cfg.copy(batchCapacity = math.max(1L, count.toLong)))
    try {
      if (init.isDefined) GpuRoundNative.loadInputs(ctx, begin, count, init.get)
      val ids = Array.tabulate(count)(i => begin + i)
      val sums = new Array[Byte](24 * count)
      val recs = new Array[Int](4 * cfg.n * count)
      GpuRoundNative.fetch(ctx, ids, sums, recs)
      recs
    } finally GpuRoundNative.destroy(ctx)
  }

  /** Run instances checking a compiled Spec (GpuSpec.compile) instead of the built-in
    * checker: fail counts per program slot (psg_run_batch_spec). */
  def runSpec(alg: Algorithm[_, _], cfg: GpuConfig, begin: Long, count: Long, prog: GpuSpec.Program,
              init: Option[Array[Int]] = None): GpuResult = {
    val id = algId(alg)
    require(prog.alg == 0 || prog.alg == id, s"the Spec program was compiled for algorithm ${prog.alg}, not $id")
    checkRange(cfg, begin, count)
    init.foreach(a => require(a.length == count * cfg.n, s"init must hold count * n = ${count * cfg.n} values"))
    val ctx = create(id, cfg)
    try {
      GpuRoundNative.loadInputs(ctx, begin, count, init.orNull)
      summary(GpuRoundNative.runBatchSpec(ctx, begin, count, prog.code, prog.slotEntry, prog.slotFlags,
        prog.termEntry, prog.nVars, prog.alg, prog.modulePath, null), cfg.rounds)
    } finally GpuRoundNative.destroy(ctx)
  }

  def run(alg: Algorithm[_, _], cfg: GpuConfig, begin: Long, count: Long, init: Option[Array[Int]] = None,
          decide: Option[(Long, Int, Int, Int) => Unit] = None): GpuResult = {
    val id = algId(alg)
    if (realValued(id)) throw new IllegalArgumentException(alg.getClass.getName + " is real-valued: use runReal")
    checkRange(cfg, begin, count)
    init.foreach(a => require(a.length == count * cfg.n, s"init must hold count * n = ${count * cfg.n} values"))
    val ctx = create(id, cfg)
    try {
      GpuRoundNative.loadInputs(ctx, begin, count, init.orNull)
      val res = summary(GpuRoundNative.runBatch(ctx, begin, count, null), cfg.rounds)
      decide.foreach { cb =>
        val cells = (count * cfg.n).toInt
        val d = new Array[Int](cells)
        val r = new Array[Int](cells)
        GpuRoundNative.copyDecisions(ctx, d, r)
        var i = 0
        while (i < cells) {
          if (r(i) >= 0) cb(begin + i / cfg.n, i % cfg.n, d(i), r(i))
          i += 1
        }
      }
      res
    } finally GpuRoundNative.destroy(ctx)
  }
}
