// GpuSpec.scala — generic Specs for the GPU checker from the JVM (SURVEY §8f rank 1).
//
// Drop into the reference build next to GpuRound.scala (src/main/scala/psync/gpu/).
// Not compiled in this repository's CI (no JVM in the image): the C side it calls,
// psg_spec_from_text (round_amd/csrc/psg_spec_text.cpp), is tested in
// tests/test_spec_text.py on texts of exactly the shape `text` below writes.
//
// A psync.Spec (psync/Specs.scala:8-16) holds Formula trees that the macros
// produced from the Scala spec code (psync/macros/FormulaExtractor.scala). `text`
// writes them as S-expressions of their own constructors (psync/formula/Formula.scala:
// Binding ForAll / Exists / Comprehension, Application(symbol, args), Variable,
// Literal); psg_spec_from_text compiles that text to the psg_spec_program bytecode,
// with the slots the Verifier would assemble (psync/verification/Verifier.scala:111-141).
package psync.gpu

import psync.Algorithm
import psync.formula._

object GpuSpec {

  /** A compiled Spec: the psg_spec_program arrays + slot names (psg.h). */
  case class Program(code: Array[Int], slotEntry: Array[Int], slotFlags: Array[Int], termEntry: Int, nVars: Int,
                     alg: Int, slotNames: Array[String], modulePath: String = null)

  /** Rounds per phase of each algorithm's Process (`rounds.length`): the `L` of the
    * roundInvariant guard (Verifier.scala:133-141). */
  val phaseLength: Map[Int, Int] = Map(1 -> 1, 2 -> 4, 3 -> 1, 4 -> 1, 5 -> 2, 6 -> 1, 7 -> 3, 8 -> 1)

  private def typeTag(t: Type): String = t match {
    case Int => "Int"
    case Bool => "Bool"
    case FSet(_) => "Set"
    case UnInterpreted("Time") => "Time"
    case _ => "pid" // psync.logic.CL.procType = UnInterpreted("ProcessID")
  }

  private def symbol(s: Symbol): String = s match {
    case Not => "Not"
    case And => "And"
    case Or => "Or"
    case Implies => "Implies"
    case Eq => "Eq"
    case Neq => "Neq"
    case Plus => "Plus"
    case Minus => "Minus"
    case Times => "Times"
    case Divides => "Divides"
    case Leq => "Leq"
    case Geq => "Geq"
    case Lt => "Lt"
    case Gt => "Gt"
    case In => "In"
    case Contains => "Contains"
    case Cardinality => "Cardinality"
    case IsDefined => "IsDefined"
    case IsEmpty => "IsEmpty"
    case Get => "Get"
    case FSome => "Some"
    case UnInterpretedFct(name, _, _) => name // fields (x, decided, __init__x, __old__x, ...), HO, coord
    case other => other.toString // e.g. ReduceTime's toInt / fromInt
  }

  /** One Formula as text. */
  def formula(f: Formula): String = f match {
    case Literal(b: Boolean) => s"(Lit $b)"
    case IntLit(i) => s"(Lit $i)"
    case Variable(name) => s"(Var $name)"
    case Binding(bt, vs, body) =>
      val head = bt match {
        case ForAll => "ForAll"
        case Exists => "Exists"
        case Comprehension => "Comprehension"
      }
      vs.map(v => s"(${v.name} ${typeTag(v.tpe)})").mkString(s"($head (", " ", s") ${formula(body)})")
    case Application(fct, args) => args.map(a => " " + formula(a)).mkString(s"(App ${symbol(fct)}", "", ")")
    case other => throw new IllegalArgumentException("no GPU lowering for " + other)
  }

  /** The whole Spec as text (the format of round_amd/formula.py "Formula text"). */
  def text(spec: Algorithm[_, _]#Spec, phase: Int): String = {
    val sb = new StringBuilder(s"(Spec (phase $phase)\n  (invariants")
    spec.invariants.foreach(f => sb ++= " " ++= formula(f))
    sb ++= ")\n  (roundInvariants"
    spec.roundInvariants.foreach(l => sb ++= l.map(formula).mkString(" (list ", " ", ")"))
    sb ++= ")\n  (properties"
    spec.properties.foreach { case (name, f) => sb ++= s""" (prop "$name" ${formula(f)})""" }
    sb ++= ")"
    spec.safetyPredicate match {
      case True() => ()
      case sp => sb ++= s"\n  (safetyPredicate ${formula(sp)})"
    }
    sb ++= ")"
    sb.toString
  }

  /** Compile `alg`'s own Spec (or any other of its Specs) for psg_run_batch_spec. `native`:
    * also lower it to gfx950 code in the library (psg_spec_compile_native, hiprtc, cached);
    * `fused` (with native): one launch that runs the rounds and checks the Spec from
    * registers; `n`: the group size the module is instantiated for (0: every size). */
  def compile(alg: Algorithm[_, _], spec: Algorithm[_, _]#Spec, native: Boolean = false, fused: Boolean = false,
              n: Int = 0): Program = {
    val id = GpuRound.algId(alg)
    val t = text(spec, phaseLength.getOrElse(id, 1))
    val packed = GpuRoundNative.compileSpec(t, id)
    val (ns, nw) = (packed(0), packed(1))
    val module = if (native || fused) GpuRoundNative.compileSpecNative(t, id, fused, n) else null
    Program(packed.slice(4, 4 + nw), packed.slice(4 + nw, 4 + nw + ns), packed.slice(4 + nw + ns, 4 + nw + 2 * ns),
            packed(2), packed(3), id, GpuRoundNative.compileSpecNames(t, id).split("\n"), module)
  }
}
