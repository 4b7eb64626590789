"""Diagnostic: build phase-ablation variants of libsrbd_mpc.so from a PATCHED COPY of csrc (the
product sources are never modified; see scripts/build_variant.py for the build flags).

    python scripts/ablate.py OUT NAME     NAME in VARIANTS below

Each variant runs one idempotent phase twice per Newton iteration, so (variant - base) is that
phase's marginal cost in the real 2-waves/SIMD context. Timing: scripts/ab_bench.sh-style runs of
bench.py with SRBD_LIB=OUT on the GPU box."""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "biped_pympc_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
REG = "pdipm_srbd_reg.hpp"


def _dup(src: str, start: str, end: str) -> str:
    a = src.index(start)
    b = src.index(end, a)
    return src[:b] + "{\n" + src[a:b] + "}\n" + src[b:]


# The S_ii build on the matrix cores (v_mfma_f64_16x16x4f64): measured 4 % SLOWER than the VALU
# build it replaces (profiles/r02/mfma_sii.txt), so it lives here as a variant, not in the product.
SII_MFMA = r'''    // S_ii = K + P Phi_u,i^-1 P^T on the matrix cores (v_mfma_f64_16x16x4f64, one wave per product):
    // P = [N_L | N_R] (12 x 8: the stage-invariant u block's foot columns, padded to 16 rows) and
    // Phi_u,i^-1 = blockdiag(Phi_L,i^-1, Phi_R,i^-1) (8 x 8). U = Phi^-1 P^T (two k-steps), then
    // S = K + P U (two k-steps) with U's accumulator registers j = 0, 1 serving directly as the
    // second product's B operand of k-step j (scripts/mfma_f64_layout.hip checks both lane maps with
    // exact data). Lane l holds P[l & 15][4 s + (l >> 4)] (the A operand of P U and, as P^T[k][col],
    // the B operand of Phi^-1 P^T: the same register) and produces S[(l >> 4) + 4 j][l & 15].
    // Wave w of a two-wave QP takes stages w, w + 2, ...
    {
      typedef double d4 __attribute__((ext_vector_type(4)));
      constexpr int NW = TPB / 64;
      const int lw = lane & 63, wv = lane >> 6, r16 = lw & 15, kq = lw >> 4;
      double pa[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int kk = 4 * s + kq;
        pa[s] = r16 < 12 ? Nd[nd_idx(r16, foot_colj(kk >> 2, kk & 3))] : 0.0;
      }
      // this lane's four S entries (row kq + 4 j, column r16): packed-slot offset and K index;
      // only the lower triangle is stored (the packed block keeps one copy of each pair)
      int sl[4], sk[4];
      bool keep[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = kq + 4 * j, c = r16;
        keep[j] = r < 12 && c < 12 && r >= c;
        const int sy = (r < 12 && c < 12) ? sym_idx(r, c) : 0;
        sk[j] = sy;
        sl[j] = c_dvslot[sy];
      }
      // Phi^-1 operand: row r16 (< 8: foot r16 >> 2), column 4 s + kq; zero across feet / padding
      int pho[2];
      bool phk[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int kk = 4 * s + kq;
        phk[s] = r16 < 8 && (r16 >> 2) == (kk >> 2);
        pho[s] = 10 * (r16 >> 2 & 1) + sym_idx(r16 & 3, kk & 3);
      }
#pragma unroll
      for (int t = 0; t < N / NW; ++t) {
        const int i = NW * t + wv;
        const double* ph_ = PHs + 20 * i;
        double ba[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const double v = ph_[pho[s]];
          ba[s] = phk[s] ? v : 0.0;
        }
        d4 u = {0.0, 0.0, 0.0, 0.0};
        u = __builtin_amdgcn_mfma_f64_16x16x4f64(ba[0], pa[0], u, 0, 0, 0);
        u = __builtin_amdgcn_mfma_f64_16x16x4f64(ba[1], pa[1], u, 0, 0, 0);
        const double* Kt = i == 0 ? K0 : K1;
        d4 acc;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = Kt[sk[j]];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[0], u[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[1], u[1], acc, 0, 0, 0);
        double* blk = DV + kDvStride * dv_pos<N>(i);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (keep[j]) blk[sl[j]] = acc[j];
      }
    }
'''


def _sii_mfma(src: str) -> str:
    a = src.index("    // S_ii = K + sum_f N_f Phi_f^-1 N_f^T in two divergence-free passes")
    b = src.index("    __syncthreads();\n    PROF_ADD(1);", a)
    return src[:a] + SII_MFMA + src[b:]


VARIANTS = {
    "sii_mfma": _sii_mfma,
    # the S_ii build (after the Phi_u foot inverses): its two entry passes and their barrier
    "sii2": lambda s: _dup(s, "    // S_ii = K + sum_f N_f Phi_f^-1 N_f^T in two divergence-free passes",
                           "    PROF_ADD(1);"),
    # one extra back-substitution pass over the refinement's QV (a chain's cost; results change)
    "chain2": lambda s: s.replace("    C.refine_rhs();\n    C.template solve_chain<false>();",
                                  "    C.refine_rhs();\n    C.template solve_chain<false>();\n    C.template solve_chain<true>();"),
    "residuals2": lambda s: s.replace("    double mu = C.residuals(it == 0);",
                                      "    (void)C.residuals(false);\n    double mu = C.residuals(it == 0);"),
    # the factor chain with the fused affine forward elimination run twice (not idempotent: the
    # second pass inverts the inverses; cost only)
    "fchain2": lambda s: s.replace("    C.template factor_chain<true>();  // + the affine forward elimination",
                                   "    C.template factor_chain<true>();\n    C.template factor_chain<true>();"),
    # the combined solve's right-hand side twice (idempotent)
    "rhs2": lambda s: s.replace("    solve_rhs<kMode>(smu, rx);\n    solve_chain<false>();",
                                "    solve_rhs<kMode>(smu, rx);\n    solve_rhs<kMode>(smu, rx);\n    solve_chain<false>();"),
    # the combined solve's finish twice (cost only)
    "finish2": lambda s: s.replace("    solve_chain<false>();\n    solve_finish<false, false, true>();",
                                   "    solve_chain<false>();\n    solve_finish<false, false, true>();\n"
                                   "    solve_finish<false, false, true>();"),
    # odd workgroups start their Newton loop ~40k cycles late (5 x s_sleep 127), so the two waves
    # sharing a SIMD tend to sit in different phases (chain vs row-parallel) -- a phase-offset probe
    "stagger": lambda s: s.replace("  PROF_MARK_CTX(C);\n",
                                   "  PROF_MARK_CTX(C);\n  if (blockIdx.x & 1) {\n"
                                   "    for (int k = 0; k < 5; ++k) __builtin_amdgcn_s_sleep(127);\n  }\n"),
    # the same without the progress-ordered wave priority (which pulls the two waves back together)
    "stagger_noprio": lambda s: s.replace("  PROF_MARK_CTX(C);\n",
                                          "  PROF_MARK_CTX(C);\n  if (blockIdx.x & 1) {\n"
                                          "    for (int k = 0; k < 5; ++k) __builtin_amdgcn_s_sleep(127);\n  }\n")
                                 .replace("#define SRBD_PROGRESS_PRIO 1", "#define SRBD_PROGRESS_PRIO 0"),
    "noprio": lambda s: s.replace("#define SRBD_PROGRESS_PRIO 1", "#define SRBD_PROGRESS_PRIO 0"),
    # the S_ii build's sparse-entry stage loop fully unrolled (the product unrolls it by 2)
    "sii_unroll": lambda s: s.replace("#pragma unroll 2\n      for (int i = wv * (N / NW);",
                                      "#pragma unroll\n      for (int i = wv * (N / NW);"),
    # the Phi_u foot-block inverses with rcp3 pivots instead of IEEE division
    "foot_rcp": lambda s: s.replace("      sweep_inverse<4>(a);  // IEEE pivots",
                                    "      sweep_inverse<4, true>(a);  // IEEE pivots"),
    # no affine refinement at degenerate iterates (the branch compiled out)
    "no_aff_ref": lambda s: s.replace("    if (degen) {  // full affine finish", "    if (false) {  // full affine finish"),
    # the refinement's residual (KKT rows 1, 4) twice (cost only)
    "refine2": lambda s: s.replace("    C.refine_rhs();\n", "    C.refine_rhs();\n    C.refine_rhs();\n"),
    # N = 20 with 11.5 KB more LDS per QP (the dense separator fills a partitioned chain would keep,
    # 10 stages x 12 x 12 doubles): 3 QPs per CU instead of 4 (occupancy cost only, same arithmetic)
    "pad20": lambda s: s.replace("total = end > former ? end : former;",
                                 "total = (end > former ? end : former) + (N == 20 ? 1440 : 0);"),
}


def build(out: str, name: str) -> str:
    with tempfile.TemporaryDirectory() as td:
        d = os.path.join(td, "biped_pympc_amd", "csrc")
        shutil.copytree(CSRC, d)
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(td, "include"))
        p = os.path.join(d, REG)
        src = open(p).read()
        new = VARIANTS[name](src)
        assert new != src, name
        open(p, "w").write(new)
        o20, om = os.path.join(td, "reg20.o"), os.path.join(td, "main.o")
        base = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", "-I", os.path.join(ROOT, "include")]
        on = os.path.join(td, "regN.o")
        trk = ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"]
        procs = [subprocess.Popen(base + trk + ["-o", o20, os.path.join(d, "srbd_reg20.hip")]),
                 subprocess.Popen(base + trk + ["-o", on, os.path.join(d, "srbd_regN.hip")]),
                 subprocess.Popen(base + ["-DSRBD_SPLIT_REG20", "-o", om, os.path.join(d, "srbd_mpc.hip")])]
        if any(p.wait() for p in procs):
            raise SystemExit(f"variant {name}: compile failed")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", out, om, o20, on], check=True)
    return out


if __name__ == "__main__":
    print(build(sys.argv[1], sys.argv[2]))
