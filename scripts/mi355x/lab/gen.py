"""Build x2lab_kernel.inc from the fused kernel in csrc/src/kernels/stencil7x2.hip: lab_base (ablation bits ABL:
1 no output stores, 2 no lookahead loads) and lab_var (the same plus the experimental transform below)."""
import os
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "../../..")
src = open(os.path.join(ROOT, "csrc/src/kernels/stencil7x2.hip")).read()
a = src.index("template <typename T, int NW, int PF, int KIND, int WRAP>\n// 12 waves")
b = src.index("// S o S on a few small boxes")
k = src[a:b]
k = k.replace("template <typename T, int NW, int PF, int KIND, int WRAP>", "template <typename T, int NW, int PF, int KIND, int WRAP, int ABL>")
k = k.replace("      load_row(z + (NC - 1) * dz, sn);", "      if (!(ABL & 2)) load_row(z + (NC - 1) * dz, sn);")
k = k.replace("        if (outRow) {", "        if (!(ABL & 1) && outRow) {")
base = k.replace("void stencil7x2_kernel(StencilArgs<T> a)", "void lab_base(StencilArgs<T> a)")
# variant: the output row of step t is stored at the start of step t+1 (after its lookahead loads), not before the
# barrier of step t
var = k.replace("void stencil7x2_kernel(StencilArgs<T> a)", "void lab_var(StencilArgs<T> a)")
old_store = var[var.index("        if (!(ABL & 1) && outRow) {"):var.index("      // 4. publish src plane")]
var = var.replace(old_store, "        Op = o;\n        zp_ = z;\n      }\n")
store_fn = old_store.replace("        if (!(ABL & 1) && outRow) {", "      if (!(ABL & 1) && outRow && zp_ >= 0) {").replace("int64_t(z)", "int64_t(zp_)").replace("= o;", "= Op;").replace("(o,", "(Op,").replace("o[e]", "Op[e]")
store_fn = store_fn.rstrip()
assert store_fn.endswith("}"), store_fn[-50:]
store_fn = store_fn[: -1].rstrip()  # drop the closing brace of `if (t >= 0) {`
var = var.replace("      if (!(ABL & 2)) load_row(z + (NC - 1) * dz, sn);", "      if (!(ABL & 2)) load_row(z + (NC - 1) * dz, sn);\n" + store_fn + "\n")
var = var.replace("    int buf = 0;\n    int t = -2;", "    int buf = 0;\n    int t = -2;\n    NV Op;\n    int zp_ = -1;")
var = var.replace("    while (run_phases(step, std::make_integer_sequence<int, NC>{})) {\n    }",
                  "    while (run_phases(step, std::make_integer_sequence<int, NC>{})) {\n    }\n    {\n      const int z = 0; (void)z;\n" + store_fn + "\n    }")
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "x2lab_kernel.inc"), "w").write(base + "\n" + var)
