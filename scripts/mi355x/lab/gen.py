"""Build x2lab_kernel.inc from csrc/src/kernels/stencil7x2.hip (the helpers come from stencil_wave.hpp): lab_col = stencil7x2_kernel and
lab_row = stencil7x2_row_kernel, each with ablation bits ABL (1: no output stores, 2: no lookahead loads)."""
import os
HERE = os.path.dirname(os.path.abspath(__file__))
src = open(os.path.join(HERE, "../../../csrc/src/kernels/stencil7x2.hip")).read()


def ablate(k):
    k = k.replace("      load_row(z + (NC - 1) * dz, sn);", "      if (!(ABL & 2)) load_row(z + (NC - 1) * dz, sn);")
    k = k.replace("        if (outRow) {", "        if (!(ABL & 1) && outRow) {")
    return k


a = src.index("template <typename T, int NW, int PF, int KIND, int WRAP>\n// 12 waves")
b = src.index("// Whole-row variant of the fused pair")
col = src[a:b].replace("template <typename T, int NW, int PF, int KIND, int WRAP>",
                       "template <typename T, int NW, int PF, int KIND, int WRAP, int ABL>")
col = ablate(col.replace("void stencil7x2_kernel(StencilArgs<T> a)", "void lab_col(StencilArgs<T> a)"))
c = src.index("template <int NW, int PF, int KIND>\n__global__")
d = src.index("// 512-cell columns (fp32)") if "// 512-cell columns (fp32)" in src else src.index("// S o S on a few small boxes")
rot = src[b:c]
row = src[c:d].replace("template <int NW, int PF, int KIND>", "template <int NW, int PF, int KIND, int ABL>")
row = ablate(row.replace("stencil7x2_row_kernel(", "lab_row("))
assert "ABL & 2" in col and "ABL & 1" in col and "ABL & 2" in row and "ABL & 1" in row
# lab_rownt: the row kernel with nontemporal loads for the rows no other block reads (waves 4..7 of 12)
old_ld = "#pragma unroll\n      for (int h = 0; h < H; ++h) C[k][h] = *reinterpret_cast<const NV *>(b + h * HS * int(sizeof(T)));"
assert old_ld in row
rownt = row.replace("lab_row(", "lab_rownt(").replace(old_ld, """      if (w >= 4 && w < 8) {
#pragma unroll
        for (int h = 0; h < H; ++h) C[k][h] = __builtin_nontemporal_load(reinterpret_cast<const NV *>(b + h * HS * int(sizeof(T))));
      } else {
#pragma unroll
        for (int h = 0; h < H; ++h) C[k][h] = *reinterpret_cast<const NV *>(b + h * HS * int(sizeof(T)));
      }""")
open(os.path.join(HERE, "x2lab_kernel.inc"), "w").write(col + "\n" + rot + "\n" + row + "\n" + rownt)
