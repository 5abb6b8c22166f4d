"""Regenerate the instrumented kernel copies in potrf_ubench.hip from the library source."""
import re
import sys

U = "scripts/ubench/potrf_ubench.hip"
LIB = "fish-eye_bundle_adjustment_amd/csrc/fba_chol.hip"
u = open(U).read()
lib = open(LIB).read()
a = lib.index("__global__ __launch_bounds__(256) void k_potrf128(")
b = lib.index("// ------------------------------------------------------------------------------------------------\n// k_trsm128:")
k = lib[a:b].replace("void k_potrf128(", "void k_potrf_ts(").replace(
    "double* __restrict__ dinv, double* __restrict__ scal) {",
    "double* __restrict__ dinv, double* __restrict__ scal, unsigned long long* ts) {\n"
    "#define T0(i) do { if (threadIdx.x == 0) ts[i] = __builtin_amdgcn_s_memtime(); } while (0)\n    T0(0);")
k = k.replace("#define AT(r, c)", "#define AT_(r, c)").replace("AT(", "AT_(").replace("#undef AT", "#undef AT_\n#undef T0")
k = k.replace("        if (wave == 0) {\n            ok = leaf_factor(a, x, lr);", "        if (wave == 0) {\n            T0(1);\n            ok = leaf_factor(a, x, lr);\n            T0(2);")
k = k.replace("        __syncthreads();  // B1: L_ss, D_s in LDS; column s updated\n", "        __syncthreads();  // B1: L_ss, D_s in LDS; column s updated\n        T0(3 + 4 * s);\n")
k = k.replace("        __syncthreads();  // B2: panel column s solved\n", "        __syncthreads();  // B2: panel column s solved\n        T0(4 + 4 * s);\n")
k = k.replace("            ok &= leaf_factor(a, x, lr);", "            T0(5 + 4 * s);\n            ok &= leaf_factor(a, x, lr);\n            T0(6 + 4 * s);")
k = k.replace("    store_col(CB / IB - 1, tid, 256);\n", "    store_col(CB / IB - 1, tid, 256);\n    __builtin_amdgcn_s_waitcnt(0);\n    __syncthreads();\n    T0(40);\n")
s0 = u.index("// instrumented copy of k_potrf128\n")
s1 = u.index("// end of instrumented copy", s0)
u = u[:s0] + "// instrumented copy of k_potrf128\n" + k + "\n" + u[s1:]
open(U, "w").write(u)
