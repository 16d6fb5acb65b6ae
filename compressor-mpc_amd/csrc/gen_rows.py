#!/usr/bin/env python3
"""Generate rows_blocks.inc: the inline-asm DPP blocks of the row-layout build
kernel (build_rows.hip; one QP per 16-lane DPP row, four QPs per wave).

  rows_chain<NS, NY, ND>(pP, pS, mP, mS, aP, aS):
      for l < NS:  aP[o] += bcast_l(pP[o]) * mP[l]   (o < NY: rows of P_r = L_W' C A^r)
                   aS    += bcast_l(pS)    * mS[l]   (free-response simulation)
      for k < ND:  aS    += bcast_{16-ND+k}(pS) * mS[NS+k]   (delayed-input carriers)
    The NY + 1 accumulation chains are interleaved link by link, so consecutive
    instructions never depend on each other.
  rows_gacc<NY, NUT, NU, M>(cv, acc):
      acc[a] += bcast_{L_a}(cv[o]) * cv[o]   for o < NY, a < NU*M,
      L_a = (a / NU) * NUT + a % NU   (gather lane of own QP column a)

Every block opens with `s_nop 1`: a VALU write of a VGPR followed by a DPP read
of it needs two wait states and hipcc does not pad inside an asm statement
(cdna_hip_programming.md §5.7).  No DPP source is written inside a block.
"""
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rows_blocks.inc")
CTRL = "row_mask:0xf bank_mask:0xf"

# (NS, NY, ND) of the chain blocks and (NY, NUT, NU, M) of the gather blocks
# used by the instantiated kernels (build_rows.hip launcher list)
CHAINS = [(11, 3, 2), (11, 2, 2), (10, 2, 2), (10, 4, 2)]
GACCS = [(3, 4, 2, 2), (2, 4, 2, 2), (3, 4, 4, 2), (4, 4, 2, 2), (4, 4, 4, 2), (3, 4, 2, 1)]
# (NS, NY, ND, NUT, NU, M) of the fused chain + gather blocks (the launcher's cases)
FUSED = [(11, 3, 2, 4, 2, 2), (11, 2, 2, 4, 2, 2), (11, 3, 2, 4, 4, 2), (10, 2, 2, 4, 2, 2),
         (10, 4, 2, 4, 2, 2), (10, 4, 2, 4, 4, 2), (11, 3, 2, 4, 2, 1)]


def chain(ns, ny, nd):
    # operands: outputs aP[0..ny-1] = %0.., aS = %ny; inputs pP, pS, mP, mS
    o_aS = ny
    i0 = ny + 1
    o_pP = [i0 + o for o in range(ny)]
    o_pS = i0 + ny
    o_mP = [o_pS + 1 + l for l in range(ns)]
    o_mS = [o_pS + 1 + ns + l for l in range(ns + nd)]
    lines = ['"s_nop 1\\n\\t"']
    for l in range(ns):
        for o in range(ny):
            lines.append(f'"v_fmac_f64_dpp %{o}, %{o_pP[o]}, %{o_mP[l]} row_newbcast:{l} {CTRL}\\n\\t"')
        lines.append(f'"v_fmac_f64_dpp %{o_aS}, %{o_pS}, %{o_mS[l]} row_newbcast:{l} {CTRL}\\n\\t"')
    for k in range(nd):
        lines.append(f'"v_fmac_f64_dpp %{o_aS}, %{o_pS}, %{o_mS[ns + k]} row_newbcast:{16 - nd + k} {CTRL}\\n\\t"')
    outs = ", ".join([f'"+v"(aP[{o}])' for o in range(ny)] + ['"+v"(aS)'])
    ins = ", ".join([f'"v"(pP[{o}])' for o in range(ny)] + ['"v"(pS)'] +
                    [f'"v"(mP[{l}])' for l in range(ns)] + [f'"v"(mS[{l}])' for l in range(ns + nd)])
    body = "\n      ".join(lines)
    return (f"template <> __device__ __forceinline__ void rows_chain<{ns}, {ny}, {nd}>("
            f"const double* pP, double pS, const double* mP, const double* mS, double* aP, double& aS) {{\n"
            f"  asm({body}\n      : {outs}\n      : {ins});\n}}\n")


def gacc(ny, nut, nu, mm):
    nv = nu * mm
    lines = ['"s_nop 1\\n\\t"']
    for o in range(ny):
        for a in range(nv):
            src = (a // nu) * nut + a % nu
            lines.append(f'"v_fmac_f64_dpp %{a}, %{nv + o}, %{nv + o} row_newbcast:{src} {CTRL}\\n\\t"')
    outs = ", ".join(f'"+v"(acc[{a}])' for a in range(nv))
    ins = ", ".join(f'"v"(cv[{o}])' for o in range(ny))
    body = "\n      ".join(lines)
    return (f"template <> __device__ __forceinline__ void rows_gacc<{ny}, {nut}, {nu}, {mm}>("
            f"const double* cv, double* acc) {{\n"
            f"  asm({body}\n      : {outs}\n      : {ins});\n}}\n")


def chain_gacc(ns, ny, nd, nut, nu, mm):
    """rows_chain and rows_gacc of one step in one block: the gather FMAs are
    spread between the chain's link groups, so 4 + nV accumulators are in
    flight instead of 4 (microbench_hybrid V3: -4 % per step at 3 waves/SIMD).
    Same FMA order per accumulator as the two separate blocks."""
    nv = nu * mm
    o_aS = ny
    o_acc = [ny + 1 + a for a in range(nv)]
    i0 = ny + 1 + nv
    o_pP = [i0 + o for o in range(ny)]
    o_pS = i0 + ny
    o_mP = [o_pS + 1 + l for l in range(ns)]
    o_mS = [o_pS + 1 + ns + l for l in range(ns + nd)]
    o_cv = [o_pS + 1 + ns + ns + nd + o for o in range(ny)]
    gl = []
    for o in range(ny):
        for a in range(nv):
            src = (a // nu) * nut + a % nu
            gl.append(f'"v_fmac_f64_dpp %{o_acc[a]}, %{o_cv[o]}, %{o_cv[o]} row_newbcast:{src} {CTRL}\\n\\t"')
    per = -(-len(gl) // ns)  # gather FMAs after each link group
    lines = ['"s_nop 1\\n\\t"']
    for l in range(ns):
        for o in range(ny):
            lines.append(f'"v_fmac_f64_dpp %{o}, %{o_pP[o]}, %{o_mP[l]} row_newbcast:{l} {CTRL}\\n\\t"')
        lines.append(f'"v_fmac_f64_dpp %{o_aS}, %{o_pS}, %{o_mS[l]} row_newbcast:{l} {CTRL}\\n\\t"')
        lines.extend(gl[l * per:(l + 1) * per])
    for k in range(nd):
        lines.append(f'"v_fmac_f64_dpp %{o_aS}, %{o_pS}, %{o_mS[ns + k]} row_newbcast:{16 - nd + k} {CTRL}\\n\\t"')
    outs = ", ".join([f'"+v"(aP[{o}])' for o in range(ny)] + ['"+v"(aS)'] + [f'"+v"(acc[{a}])' for a in range(nv)])
    ins = ", ".join([f'"v"(pP[{o}])' for o in range(ny)] + ['"v"(pS)'] +
                    [f'"v"(mP[{l}])' for l in range(ns)] + [f'"v"(mS[{l}])' for l in range(ns + nd)] +
                    [f'"v"(cv[{o}])' for o in range(ny)])
    body = "\n      ".join(lines)
    return (f"template <> __device__ __forceinline__ void rows_chain_gacc<{ns}, {ny}, {nd}, {nut}, {nu}, {mm}>("
            f"const double* pP, double pS, const double* mP, const double* mS, double* aP, double& aS, "
            f"const double* cv, double* acc) {{\n"
            f"  asm({body}\n      : {outs}\n      : {ins});\n}}\n")


SPLITS = [3, 5, 7]  # leading chain link groups of rows_chain_head (CMPC_ROWS_SPLIT)


def chain_head(ns, ny, nd, split):
    """The first `split` link groups of rows_chain (no gather FMAs): the
    running sums of the gather columns, which consume the LDS reads of the
    previous step, then run after them instead of at the start of the step,
    so the wave does not wait on that LDS round trip (round 3)."""
    o_aS = ny
    i0 = ny + 1
    o_pP = [i0 + o for o in range(ny)]
    o_pS = i0 + ny
    o_mP = [o_pS + 1 + l for l in range(split)]
    o_mS = [o_pS + 1 + split + l for l in range(split)]
    lines = ['"s_nop 1\\n\\t"']
    for l in range(split):
        for o in range(ny):
            lines.append(f'"v_fmac_f64_dpp %{o}, %{o_pP[o]}, %{o_mP[l]} row_newbcast:{l} {CTRL}\\n\\t"')
        lines.append(f'"v_fmac_f64_dpp %{o_aS}, %{o_pS}, %{o_mS[l]} row_newbcast:{l} {CTRL}\\n\\t"')
    outs = ", ".join([f'"+v"(aP[{o}])' for o in range(ny)] + ['"+v"(aS)'])
    ins = ", ".join([f'"v"(pP[{o}])' for o in range(ny)] + ['"v"(pS)'] +
                    [f'"v"(mP[{l}])' for l in range(split)] + [f'"v"(mS[{l}])' for l in range(split)])
    body = "\n      ".join(lines)
    return (f"template <> __device__ __forceinline__ void rows_chain_head<{ns}, {ny}, {nd}, {split}>("
            f"const double* pP, double pS, const double* mP, const double* mS, double* aP, double& aS) {{\n"
            f"  asm({body}\n      : {outs}\n      : {ins});\n}}\n")


def chain_gacc_tail(ns, ny, nd, nut, nu, mm, split):
    """Link groups split .. ns-1 and the carriers of rows_chain with every
    gather FMA of the step spread between them (same FMA order per
    accumulator as rows_chain_gacc)."""
    nv = nu * mm
    o_aS = ny
    o_acc = [ny + 1 + a for a in range(nv)]
    i0 = ny + 1 + nv
    o_pP = [i0 + o for o in range(ny)]
    o_pS = i0 + ny
    nl = ns - split
    o_mP = [o_pS + 1 + l for l in range(nl)]
    o_mS = [o_pS + 1 + nl + l for l in range(nl + nd)]
    o_cv = [o_pS + 1 + nl + nl + nd + o for o in range(ny)]
    gl = []
    for o in range(ny):
        for a in range(nv):
            src = (a // nu) * nut + a % nu
            gl.append(f'"v_fmac_f64_dpp %{o_acc[a]}, %{o_cv[o]}, %{o_cv[o]} row_newbcast:{src} {CTRL}\\n\\t"')
    per = -(-len(gl) // nl)
    lines = ['"s_nop 1\\n\\t"']
    for i in range(nl):
        l = split + i
        for o in range(ny):
            lines.append(f'"v_fmac_f64_dpp %{o}, %{o_pP[o]}, %{o_mP[i]} row_newbcast:{l} {CTRL}\\n\\t"')
        lines.append(f'"v_fmac_f64_dpp %{o_aS}, %{o_pS}, %{o_mS[i]} row_newbcast:{l} {CTRL}\\n\\t"')
        lines.extend(gl[i * per:(i + 1) * per])
    for k in range(nd):
        lines.append(f'"v_fmac_f64_dpp %{o_aS}, %{o_pS}, %{o_mS[nl + k]} row_newbcast:{16 - nd + k} {CTRL}\\n\\t"')
    outs = ", ".join([f'"+v"(aP[{o}])' for o in range(ny)] + ['"+v"(aS)'] + [f'"+v"(acc[{a}])' for a in range(nv)])
    ins = ", ".join([f'"v"(pP[{o}])' for o in range(ny)] + ['"v"(pS)'] +
                    [f'"v"(mP[{split + i}])' for i in range(nl)] +
                    [f'"v"(mS[{split + i}])' for i in range(nl)] +
                    [f'"v"(mS[{ns + k}])' for k in range(nd)] +
                    [f'"v"(cv[{o}])' for o in range(ny)])
    body = "\n      ".join(lines)
    return (f"template <> __device__ __forceinline__ void rows_chain_gacc_tail<{ns}, {ny}, {nd}, {nut}, {nu}, {mm}, {split}>("
            f"const double* pP, double pS, const double* mP, const double* mS, double* aP, double& aS, "
            f"const double* cv, double* acc) {{\n"
            f"  asm({body}\n      : {outs}\n      : {ins});\n}}\n")


def main():
    parts = ["// Generated by gen_rows.py — do not edit.\n",
             "template <int NS, int NY, int ND> __device__ __forceinline__ void rows_chain("
             "const double*, double, const double*, const double*, double*, double&);\n",
             "template <int NY, int NUT, int NU, int M> __device__ __forceinline__ void rows_gacc("
             "const double*, double*);\n"]
    for c in CHAINS:
        parts.append(chain(*c))
    for g in GACCS:
        parts.append(gacc(*g))
    parts.append("template <int NS, int NY, int ND, int NUT, int NU, int M> __device__ __forceinline__ void "
                 "rows_chain_gacc(const double*, double, const double*, const double*, double*, double&, "
                 "const double*, double*);\n")
    for c in FUSED:
        parts.append(chain_gacc(*c))
    parts.append("template <int NS, int NY, int ND, int SPLIT> __device__ __forceinline__ void "
                 "rows_chain_head(const double*, double, const double*, const double*, double*, double&);\n")
    parts.append("template <int NS, int NY, int ND, int NUT, int NU, int M, int SPLIT> __device__ __forceinline__ "
                 "void rows_chain_gacc_tail(const double*, double, const double*, const double*, double*, "
                 "double&, const double*, double*);\n")
    heads = sorted({(c[0], c[1], c[2]) for c in FUSED})
    for sp in SPLITS:
        for h in heads:
            parts.append(chain_head(*h, sp))
        for c in FUSED:
            parts.append(chain_gacc_tail(*c, sp))
    with open(OUT, "w") as fh:
        fh.write("\n".join(parts))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
