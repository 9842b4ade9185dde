// HoHarness.scala — in-JVM lockstep HO harness over the reference's own rounds
// (SURVEY §8c: "a ~200-LoC Scala harness in package psync can drive RtProcess
// directly ... confirm the CHAMP tie-break assumption and the coin convention").
//
// Drop into the reference build next to GpuRound.scala (package psync.gpu, so the
// protected[psync] members of RtProcess are visible). Not compiled in this
// repository (no JVM in the image).
//
// It executes ONE instance with the reference's Process / Round code — no netty,
// no Kryo, no InstanceHandler — under HO sets taken from the GPU library
// (GpuRound.materialize = psg_materialize_schedule, or a counterexample file's
// HO section), with exactly the build's lockstep semantics (DESIGN.md §2):
//   round k: every non-halted process runs `init()` (psync/Process.scala:67-70);
//   messages come from the pre-state via the round's public `send()`
//   (psync/Round.scala:89-91); q's message reaches p iff q is in HO(p, k), q is not
//   halted and p is in dom(send_q), delivered by the round's public `receive`
//   in ascending q (so `mailbox` is built by Scala's own immutable.Map, i.e. the
//   CHAMP iteration order the GPU emulates); then `update(didTimeout)`
//   (psync/Process.scala:80-82) runs `Round.update(mailbox)`; `false` =
//   exitAtEndOfRound (psync/Round.scala:42-55).
// BenOr's coin: before each R1 update the harness seeds scala.util.Random with
// s = Philox4x32-10(seed, instance, k, pid | 0x8000 << 16) word 0 (SURVEY §8a A8).
// The per-process results (decision, decision round, halt round) are compared
// with GpuRound.records (psg_fetch_instances) for a sampled subset of ids.
package psync.gpu

import psync._
import psync.runtime.{Group, Replica}
import example.ConsensusIO

object HoHarness {

  final case class ProcResult(decision: Option[Any], decisionRound: Int, haltRound: Int)

  /** Philox4x32-10 (Random123), the build's counter-based generator (DESIGN.md §3). */
  def philox(c: Array[Int], k0: Int, k1: Int): Array[Int] = {
    var c0 = c(0); var c1 = c(1); var c2 = c(2); var c3 = c(3)
    var a = k0; var b = k1
    var i = 0
    while (i < 10) {
      val p0 = (0xD2511F53L & 0xFFFFFFFFL) * (c0 & 0xFFFFFFFFL)
      val p1 = (0xCD9E8D57L & 0xFFFFFFFFL) * (c2 & 0xFFFFFFFFL)
      val n0 = (p1 >>> 32).toInt ^ c1 ^ a
      val n2 = (p0 >>> 32).toInt ^ c3 ^ b
      c1 = p1.toInt; c3 = p0.toInt; c0 = n0; c2 = n2
      a += 0x9E3779B9; b += 0xBB67AE85
      i += 1
    }
    Array(c0, c1, c2, c3)
  }

  /** Word 0 of stream (inst, round, pid | tag): the 64-bit value s the BenOr coin seeds with. */
  def coinSeed(seed: Long, inst: Long, k: Int, pid: Int): Long = {
    val o = philox(Array(inst.toInt, (inst >>> 32).toInt, k, pid | (0x8000 << 16)), seed.toInt, (seed >>> 32).toInt)
    (o(0) & 0xFFFFFFFFL) | (o(1).toLong << 32)
  }

  private def hears(ho: Array[Long], base: Int, n: Int, W: Int, k: Int, p: Int, q: Int): Boolean =
    ((ho(base + (k * n + p) * W + (q >> 6)) >>> (q & 63)) & 1L) != 0L

  /** Run instance `inst` of `alg` for `rounds` rounds. `ho` holds [count][R][n][W] words of which this
    * instance is row `row`; `mkIO(pid, decide)` builds the process's IO (initial value + a decide
    * callback that must call `decide(value)`); `benorSeed` enables the coin convention. */
  def run[IO, P <: Process[IO]](alg: Algorithm[IO, P], n: Int, rounds: Int, inst: Long, ho: Array[Long], row: Int,
                                mkIO: (Int, Any => Unit) => IO, benorSeed: Option[Long] = None): Array[ProcResult] = {
    val W = (n + 63) / 64
    val base = row * rounds * n * W
    val reps = Array.tabulate(n)(i => Replica(new ProcessID(i.toShort), "127.0.0.1", 20000 + i))
    val decision = Array.fill[Option[Any]](n)(None)
    val decRound = Array.fill(n)(-1)
    val haltRound = Array.fill(n)(-1)
    var k = 0
    val procs: Array[P] = Array.tabulate(n) { i =>
      val p = alg.process
      p.setGroup(new Group(new ProcessID(i.toShort), reps, 0))
      p.init(mkIO(i, v => if (decision(i).isEmpty) { decision(i) = Some(v); decRound(i) = k }))
      p.asInstanceOf[P]
    }
    val halted = Array.fill(n)(false)
    val L = procs(0).rounds.length
    while (k < rounds) {
      val live = (0 until n).filter(p => !halted(p))
      if (live.nonEmpty) {
        live.foreach(p => procs(p).init())                     // incrementRound + round init
        val slot = k % L
        def round(p: Int) = procs(p).rounds(slot)._1.asInstanceOf[EventRound[Any]]
        val out: Array[Map[ProcessID, Any]] = Array.tabulate(n)(q => if (halted(q)) Map.empty else round(q).send())
        for (p <- live; q <- 0 until n if !halted(q) && hears(ho, base, n, W, k, p, q))
          out(q).get(new ProcessID(p.toShort)).foreach(m => round(p).receive(new ProcessID(q.toShort), m))
        for (p <- live) {
          if (benorSeed.isDefined && slot == 1) scala.util.Random.setSeed(coinSeed(benorSeed.get, inst, k, p))
          if (!procs(p).update(true)) { halted(p) = true; haltRound(p) = k }
        }
      }
      k += 1
    }
    Array.tabulate(n)(p => ProcResult(decision(p), decRound(p), haltRound(p)))
  }

  /** Sampled parity: the reference's own rounds in the JVM vs the GPU records, for instances
    * [begin, begin+count) of an Int consensus algorithm: the seeded schedule, the given initial
    * values ([count][n]) on both sides. Returns the ids whose per-process (decision, decision
    * round, halt round) differ. */
  def compareWithGpu[P <: Process[ConsensusIO[Int]]](alg: Algorithm[ConsensusIO[Int], P], cfg: GpuConfig,
                                                    begin: Long, count: Int, initValues: Array[Int]): Seq[Long] = {
    val (ho, _) = GpuRound.materialize(alg, cfg, begin, count)
    val recs = GpuRound.records(alg, cfg, begin, count, Some(initValues))
    val coin = if (GpuRound.algId(alg) == 5) Some(cfg.seed) else None
    (0 until count).filter { i =>
      val res = run[ConsensusIO[Int], P](alg, cfg.n, cfg.rounds, begin + i, ho, i, (pid, cb) =>
        new ConsensusIO[Int] {
          val initialValue = initValues(i * cfg.n + pid)
          def decide(value: Int): Unit = cb(value)
        }, coin)
      (0 until cfg.n).exists { p =>
        val r = (i * cfg.n + p) * 4
        val gpuDec = if (recs(r + 1) >= 0) Some(recs(r)) else None
        res(p).decision.map(_.asInstanceOf[Int]) != gpuDec || res(p).decisionRound != recs(r + 1) ||
          res(p).haltRound != recs(r + 2)
      }
    }.map(i => begin + i)
  }
}
