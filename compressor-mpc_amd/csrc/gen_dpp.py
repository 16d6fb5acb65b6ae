#!/usr/bin/env python3
"""Generate dpp_blocks.inc: inline-asm blocks of v_fmac_f64_dpp with
row_newbcast (gfx950 64-bit DPP: broadcast lane l of each 16-lane row).

hipcc does not fuse __builtin_amdgcn_mov_dpp into v_fmac_f64 for 64-bit
operands (it emits v_mov_b64_dpp + v_fmac_f64, doubling the VALU count), so
the hot loops use these blocks.  Each block opens with `s_nop 1`: a VALU
write of a VGPR followed by a DPP read of it needs 2 wait states, and hipcc
does not pad inside an asm statement (cdna_hip_programming.md §5.7 item 2).
The DPP sources of a block are never written inside it.

  prop_dpp<NS>(p, m, a0, a1):  a{l&1} += bcast_l(p) * m[l], l = 0..NS-1
  accum_dpp<LB, NU, M>(v, acc): acc[a][k] += bcast_{LB + a%NU}(v[a/NU]) * v[k]
                                 for a < NU*M, k < M
  prop1w_dpp<NS, ND>(p, m, a): prop1 over lanes 0..NS-1, then lanes 16-ND..15 with m[NS..]
  prop{3,4}w_dpp<NS, ND>(p, m, a[]): prop1w with link i into a[i % n] (n chains)
  gacc_dpp<NUT, NU, M>(v, acc): acc[a] += bcast_{(a/NU)*NUT + a%NU}(v) * v, a < NU*M
                                 (gather layout: lane k*NUT + c holds QP column (move k, input c))
"""
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dpp_blocks.inc")
CTRL = "row_mask:0xf bank_mask:0xf"


def prop(ns):
    lines = ['"s_nop 1\\n\\t"']
    for l in range(ns):
        acc = "%0" if l % 2 == 0 else "%1"
        lines.append(f'"v_fmac_f64_dpp {acc}, %2, %{3 + l} row_newbcast:{l} {CTRL}\\n\\t"')
    ins = ", ".join(['"v"(p)'] + [f'"v"(m[{l}])' for l in range(ns)])
    body = "\n      ".join(lines)
    return (f"template <> __device__ __forceinline__ void prop_dpp<{ns}>(double p, const double* m,"
            f" double& a0, double& a1) {{\n"
            f"  asm({body}\n      : \"+v\"(a0), \"+v\"(a1)\n      : {ins});\n}}\n")


def prop1(ns):
    """single accumulator chain: a += bcast_l(p) * m[l], l = 0..NS-1"""
    lines = ['"s_nop 1\\n\\t"']
    for l in range(ns):
        lines.append(f'"v_fmac_f64_dpp %0, %1, %{2 + l} row_newbcast:{l} {CTRL}\\n\\t"')
    ins = ", ".join(['"v"(p)'] + [f'"v"(m[{l}])' for l in range(ns)])
    body = "\n      ".join(lines)
    return (f"template <> __device__ __forceinline__ void prop1_dpp<{ns}>(double p, const double* m,"
            f" double& a) {{\n"
            f"  asm({body}\n      : \"+v\"(a)\n      : {ins});\n}}\n")


def prop1w(ns, nd):
    """a += bcast_l(p) * m[l] for l < NS, then a += bcast_{16-ND+k}(p) * m[NS+k]"""
    lines = ['"s_nop 1\\n\\t"']
    for l in range(ns):
        lines.append(f'"v_fmac_f64_dpp %0, %1, %{2 + l} row_newbcast:{l} {CTRL}\\n\\t"')
    for k in range(nd):
        lines.append(f'"v_fmac_f64_dpp %0, %1, %{2 + ns + k} row_newbcast:{16 - nd + k} {CTRL}\\n\\t"')
    ins = ", ".join(['"v"(p)'] + [f'"v"(m[{l}])' for l in range(ns + nd)])
    body = "\n      ".join(lines)
    return (f"template <> __device__ __forceinline__ void prop1w_dpp<{ns}, {nd}>(double p, const double* m,"
            f" double& a) {{\n"
            f"  asm({body}\n      : \"+v\"(a)\n      : {ins});\n}}\n")


def prop1w_gacc(ns, nd, nut, nu, mm):
    """prop1w chain on a with the nu*mm gather FMAs (acc[a] += bcast(v)*v)
    interleaved after the first chain links (independent work in the
    dependent chain's latency shadow)."""
    nv = nu * mm
    # operands: %0 a, %1..%nv acc, then p, v, m[0..ns+nd-1]
    P_, V_ = 1 + nv, 2 + nv
    M0 = 3 + nv
    chain = [f'"v_fmac_f64_dpp %0, %{P_}, %{M0 + l} row_newbcast:{l} {CTRL}\\n\\t"' for l in range(ns)]
    chain += [f'"v_fmac_f64_dpp %0, %{P_}, %{M0 + ns + k} row_newbcast:{16 - nd + k} {CTRL}\\n\\t"'
              for k in range(nd)]
    g = [f'"v_fmac_f64_dpp %{1 + a}, %{V_}, %{V_} row_newbcast:{(a // nu) * nut + a % nu} {CTRL}\\n\\t"'
         for a in range(nv)]
    lines = ['"s_nop 1\\n\\t"']
    gi = 0
    for i, c in enumerate(chain):
        lines.append(c)
        if gi < len(g) and i % 2 == 0:
            lines.append(g[gi]); gi += 1
    lines += g[gi:]
    outs = ", ".join(['"+v"(a)'] + [f'"+v"(acc[{a}])' for a in range(nv)])
    ins = ", ".join(['"v"(p)', '"v"(v)'] + [f'"v"(m[{l}])' for l in range(ns + nd)])
    body = "\n      ".join(lines)
    return (f"template <> __device__ __forceinline__ void prop1w_gacc_dpp<{ns}, {nd}, {nut}, {nu}, {mm}>("
            f"double p, const double* m, double& a, double v, double* acc) {{\n"
            f"  asm({body}\n      : {outs}\n      : {ins});\n}}\n")


def prop2w(ns, nd):
    """two accumulator chains (a0 even links, a1 odd links)"""
    links = [(l, f"{l}") for l in range(ns)] + [(ns + k, f"{16 - nd + k}") for k in range(nd)]
    lines = ['"s_nop 1\\n\\t"']
    for i, (mi, lane) in enumerate(links):
        acc = "%0" if i % 2 == 0 else "%1"
        lines.append(f'"v_fmac_f64_dpp {acc}, %2, %{3 + mi} row_newbcast:{lane} {CTRL}\\n\\t"')
    ins = ", ".join(['"v"(p)'] + [f'"v"(m[{l}])' for l in range(ns + nd)])
    body = "\n      ".join(lines)
    return (f"template <> __device__ __forceinline__ void prop2w_dpp<{ns}, {nd}>(double p, const double* m,"
            f" double& a0, double& a1) {{\n"
            f"  asm({body}\n      : \"+v\"(a0), \"+v\"(a1)\n      : {ins});\n}}\n")


def propnw(ns, nd, na):
    """na accumulator chains (link i into a_{i mod na}): a dependent chain of
    about (ns + nd) / na links, for waves that have no other wave on their
    SIMD to hide the FP64 latency (small batches)"""
    links = [(l, f"{l}") for l in range(ns)] + [(ns + k, f"{16 - nd + k}") for k in range(nd)]
    lines = ['"s_nop 1\\n\\t"']
    for i, (mi, lane) in enumerate(links):
        lines.append(f'"v_fmac_f64_dpp %{i % na}, %{na}, %{na + 1 + mi} row_newbcast:{lane} {CTRL}\\n\\t"')
    outs = ", ".join(f'"+v"(a[{k}])' for k in range(na))
    ins = ", ".join(['"v"(p)'] + [f'"v"(m[{l}])' for l in range(ns + nd)])
    body = "\n      ".join(lines)
    return (f"template <> __device__ __forceinline__ void prop{na}w_dpp<{ns}, {nd}>(double p, const double* m,"
            f" double* a) {{\n"
            f"  asm({body}\n      : {outs}\n      : {ins});\n}}\n")


def accum(lb, nu, mm):
    """acc is double[NU*M][M] flattened as acc[a*M + k]."""
    nv = nu * mm
    n_out = nv * mm
    groups = []
    # split into blocks of <= 24 outputs (asm operand limit 30)
    per = max(1, 24 // mm)
    a = 0
    while a < nv:
        groups.append(list(range(a, min(nv, a + per))))
        a += per
    out = [f"template <> __device__ __forceinline__ void accum_dpp<{lb}, {nu}, {mm}>("
           f"const double* v, double* acc) {{"]
    for g in groups:
        lines = ['"s_nop 1\\n\\t"']
        outs, opn = [], 0
        for aa in g:
            for k in range(mm):
                outs.append(f'"+v"(acc[{aa * mm + k}])')
        nouts = len(outs)
        idx = 0
        for aa in g:
            ka, ca = aa // nu, aa % nu
            for k in range(mm):
                src0 = nouts + ka      # v[ka] operand index
                src1 = nouts + k       # v[k]
                lines.append(f'"v_fmac_f64_dpp %{idx}, %{src0}, %{src1} '
                             f'row_newbcast:{lb + ca} {CTRL}\\n\\t"')
                idx += 1
        ins = ", ".join(f'"v"(v[{k}])' for k in range(mm))
        body = "\n      ".join(lines)
        out.append(f"  asm({body}\n      : {', '.join(outs)}\n      : {ins});")
    out.append("}\n")
    return "\n".join(out)


def gacc(nut, nu, mm):
    nv = nu * mm
    lines = ['"s_nop 1\\n\\t"']
    for a in range(nv):
        src = (a // nu) * nut + a % nu
        lines.append(f'"v_fmac_f64_dpp %{a}, %{nv}, %{nv} row_newbcast:{src} {CTRL}\\n\\t"')
    outs = ", ".join(f'"+v"(acc[{a}])' for a in range(nv))
    body = "\n      ".join(lines)
    return (f"template <> __device__ __forceinline__ void gacc_dpp<{nut}, {nu}, {mm}>(double v, double* acc) {{\n"
            f"  asm({body}\n      : {outs}\n      : \"v\"(v));\n}}\n")


def main():
    parts = ["// Generated by gen_dpp.py — do not edit.\n#pragma once\n",
             "template <int NS> __device__ __forceinline__ void prop_dpp(double, const double*,"
             " double&, double&);\n",
             "template <int LB, int NU, int M> __device__ __forceinline__ void accum_dpp("
             "const double*, double*);\n",
             "template <int NS> __device__ __forceinline__ void prop1_dpp(double, const double*,"
             " double&);\n",
             "template <int NUT, int NU, int M> __device__ __forceinline__ void gacc_dpp(double,"
             " double*);\n",
             "template <int NS, int ND> __device__ __forceinline__ void prop1w_dpp(double, const double*,"
             " double&);\n",
             "template <int NS, int ND> __device__ __forceinline__ void prop2w_dpp(double, const double*,"
             " double&, double&);\n",
             "template <int NS, int ND> __device__ __forceinline__ void prop3w_dpp(double, const double*,"
             " double*);\n",
             "template <int NS, int ND> __device__ __forceinline__ void prop4w_dpp(double, const double*,"
             " double*);\n",
             "template <int NS, int ND, int NUT, int NU, int M> __device__ __forceinline__ void "
             "prop1w_gacc_dpp(double, const double*, double&, double, double*);\n"]
    for ns in range(2, 16):
        parts.append(prop(ns))
        parts.append(prop1(ns))
        for nd in (1, 2, 3, 4):
            if ns + nd <= 16:
                parts.append(prop1w(ns, nd))
                parts.append(prop2w(ns, nd))
                parts.append(propnw(ns, nd, 3))
                parts.append(propnw(ns, nd, 4))
    # LB = NS (first Markov lane): the instantiated plants have NS = 10, 11
    for lb in (10, 11):
        for nu in (1, 2, 4):
            for mm in (1, 2, 3):
                parts.append(accum(lb, nu, mm))
    for nut in (2, 3, 4, 5, 6, 7, 8):
        for nu in range(1, nut + 1):
            for mm in (1, 2, 3):
                if mm * nut + 1 <= 16 and nu * mm <= 8:
                    parts.append(gacc(nut, nu, mm))
    # fused chain + gather accumulation for the instantiated build kernels
    for ns, nd, nut, nu, mm in [(11, 2, 4, 2, 2), (11, 2, 4, 4, 2), (10, 2, 4, 2, 2), (10, 2, 4, 4, 2),
                                (11, 2, 4, 2, 1), (11, 2, 4, 2, 3)]:
        parts.append(prop1w_gacc(ns, nd, nut, nu, mm))
    with open(OUT, "w") as fh:
        fh.write("\n".join(parts))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
