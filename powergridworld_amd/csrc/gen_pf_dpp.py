#!/usr/bin/env python3
"""Generate pgw_pf_dpp.inc: the DPP-broadcast asm groups of the power-flow solve.

The PF kernels keep the shared operand block resident in VGPRs, 16 entries per
register pair (entry e in lane e % 16 of every 16-lane row of pair e // 16), and
feed each entry to its FMA with `row_newbcast:(e % 16)`.  The scaled matrix
W''_ik = W_ik / (vb_i vb_k) is complex symmetric, so only its upper triangle is
resident (three real parts: Re, Im, Re + Im).  The lane index must be
an immediate, so every group is spelled out here per padded element count M.

Hazard rule (CDNA3/4): a VALU write of a VGPR followed by a DPP read of it needs
2 wait states, and hipcc pads nothing inside an asm string.  Each group
therefore opens with `s_nop 1`: whatever the compiler did right before the group
(a reload of a resident pair from an AGPR, the producer of x) is covered, and
inside the group the sources are read-only.  Outputs written by a movs-only
group are early-clobber so they never share a register with a source.

Usage: python3 gen_pf_dpp.py > pgw_pf_dpp.inc   (run by the Makefile)
"""
import sys

SIZES = (8, 14, 16)
DPP = "row_mask:0xf bank_mask:0xf"


def pairs_of(entries):
    ps = sorted({e // 16 for e in entries})
    return ps, {p: i for i, p in enumerate(ps)}


def asm_stmt(lines, outs, ins):
    body = "".join('      "%s\\n"\n' % ln for ln in ["s_nop 1"] + lines)
    return ("  asm(\n%s      : %s\n      : %s);\n" % (body, ", ".join(outs), ", ".join(ins)))


def tri(M, i, k):
    """Index of (i, k) in the row-major upper triangle of a symmetric M x M matrix."""
    i, k = min(i, k), max(i, k)
    return i * M - i * (i - 1) // 2 + (k - i)


def block_layout(M):
    t = M * (M + 1) // 2
    u0re = 3 * t
    g0re = u0re + 6 * M
    return dict(tri=t, u0re=u0re, u0im=u0re + M, u0sum=u0re + 2 * M, lo2=u0re + 3 * M,
                mn2=u0re + 4 * M, mx2=u0re + 5 * M, g0re=g0re, g0im=g0re + M,
                v0re=g0re + 2 * M, v0im=g0re + 2 * M + 1, size=g0re + 2 * M + 2)


def gen_node0(M, nr):
    """(vr, vi) = V0' + sum_k G'_k I'_k for output node 0 (pu, resident row)."""
    L = block_layout(M)
    ents = [L["v0re"], L["v0im"]] + [L["g0re"] + k for k in range(M)] + [L["g0im"] + k for k in range(M)]
    ps, pidx = pairs_of(ents)
    w = lambda e: "%%%d" % (2 + pidx[e // 16])
    ir = lambda k: "%%%d" % (2 + len(ps) + k)
    ii = lambda k: "%%%d" % (2 + len(ps) + M + k)
    lines = ["v_mov_b64_dpp %%0, %s row_newbcast:%d %s" % (w(L["v0re"]), L["v0re"] % 16, DPP),
             "v_mov_b64_dpp %%1, %s row_newbcast:%d %s" % (w(L["v0im"]), L["v0im"] % 16, DPP)]
    for k in range(M):             # vr and vi chains alternate (in order per chain)
        gr, gi = L["g0re"] + k, L["g0im"] + k
        lines += ["v_fmac_f64_dpp %%0, %s, %s row_newbcast:%d %s" % (w(gr), ir(k), gr % 16, DPP),
                  "v_fmac_f64_dpp %%1, %s, %s row_newbcast:%d %s" % (w(gr), ii(k), gr % 16, DPP),
                  "v_fmac_f64_dpp %%0, -%s, %s row_newbcast:%d %s" % (w(gi), ii(k), gi % 16, DPP),
                  "v_fmac_f64_dpp %%1, %s, %s row_newbcast:%d %s" % (w(gi), ir(k), gi % 16, DPP)]
    outs = ['"=&v"(vr)', '"=&v"(vi)']
    ins = ['"v"(w[%d])' % p for p in ps] + ['"v"(ir[%d])' % k for k in range(M)] + \
          ['"v"(ii[%d])' % k for k in range(M)]
    return ("template <> __device__ __forceinline__ void pf_node0<%d>(\n"
            "    double& vr, double& vi, const double (&w)[%d], const double (&ir)[%d],\n"
            "    const double (&ii)[%d]) {\n%s}\n" % (M, nr, M, M, asm_stmt(lines, outs, ins)))


def gen_column(M, k):
    """A[i] += Wr[i][k] ir ; B[i] += Wi[i][k] ii ; C[i] += (Wr+Wi)[i][k] is  (W symmetric:
    part c of entry (i, k) is block entry c * tri + tri(i, k))."""
    T = block_layout(M)["tri"]
    ents = [c * T + tri(M, i, k) for c in range(3) for i in range(M)]
    ps, pidx = pairs_of(ents)
    n_out = 3 * M
    xs = n_out + len(ps)              # operand index of ir, ii, is
    lines = []
    for c in range(3):
        for i in range(M):
            e = c * T + tri(M, i, k)
            lines.append("v_fmac_f64_dpp %%%d, %%%d, %%%d row_newbcast:%d %s"
                         % (c * M + i, n_out + pidx[e // 16], xs + c, e % 16, DPP))
    outs = ['"+v"(A[%d])' % i for i in range(M)] + ['"+v"(B[%d])' % i for i in range(M)] + \
           ['"+v"(C[%d])' % i for i in range(M)]
    ins = ['"v"(w[%d])' % p for p in ps] + ['"v"(ir)', '"v"(ii)', '"v"(is)']
    return ("template <> __device__ __forceinline__ void pf_column<%d, %d>(\n"
            "    double (&A)[%d], double (&B)[%d], double (&C)[%d], const double (&w)[%d],\n"
            "    double ir, double ii, double is) {\n%s}\n"
            % (M, k, M, M, M, (block_layout(M)["size"] + 15) // 16, asm_stmt(lines, outs, ins)))


def gen_column_v(M, k):
    """pf_column<M, K> plus the output-node-0 accumulation of the same column:
    vr += G'r_k ir - G'i_k ii ; vi += G'r_k ii + G'i_k ir (the op order of
    pf_node0, so the in-loop row equals the row evaluated after the loop)."""
    L = block_layout(M)
    T = L["tri"]
    gr, gi = L["g0re"] + k, L["g0im"] + k
    ents = [c * T + tri(M, i, k) for c in range(3) for i in range(M)] + [gr, gi]
    ps, pidx = pairs_of(ents)
    n_out = 3 * M + 2
    xs = n_out + len(ps)              # operand index of ir, ii, is
    w = lambda e: "%%%d" % (n_out + pidx[e // 16])
    lines = []
    for c in range(3):
        for i in range(M):
            e = c * T + tri(M, i, k)
            lines.append("v_fmac_f64_dpp %%%d, %s, %%%d row_newbcast:%d %s"
                         % (c * M + i, w(e), xs + c, e % 16, DPP))
    vr, vi, ir, ii = "%%%d" % (3 * M), "%%%d" % (3 * M + 1), "%%%d" % xs, "%%%d" % (xs + 1)
    node = ["v_fmac_f64_dpp %s, %s, %s row_newbcast:%d %s" % (vr, w(gr), ir, gr % 16, DPP),
            "v_fmac_f64_dpp %s, %s, %s row_newbcast:%d %s" % (vi, w(gr), ii, gr % 16, DPP),
            "v_fmac_f64_dpp %s, -%s, %s row_newbcast:%d %s" % (vr, w(gi), ii, gi % 16, DPP),
            "v_fmac_f64_dpp %s, %s, %s row_newbcast:%d %s" % (vi, w(gi), ir, gi % 16, DPP)]
    # the node-0 FMAs spread through the independent accumulations (in order
    # per chain), so no dependent FMA issues right behind its producer
    step = len(lines) // 4
    for j in reversed(range(4)):
        lines.insert(step * j + step // 2, node[j])
    outs = ['"+v"(A[%d])' % i for i in range(M)] + ['"+v"(B[%d])' % i for i in range(M)] + \
           ['"+v"(C[%d])' % i for i in range(M)] + ['"+v"(vr)', '"+v"(vi)']
    ins = ['"v"(w[%d])' % p for p in ps] + ['"v"(ir)', '"v"(ii)', '"v"(is)']
    return ("template <> __device__ __forceinline__ void pf_column_v<%d, %d>(\n"
            "    double (&A)[%d], double (&B)[%d], double (&C)[%d], double& vr, double& vi,\n"
            "    const double (&w)[%d], double ir, double ii, double is) {\n%s}\n"
            % (M, k, M, M, M, (L["size"] + 15) // 16, asm_stmt(lines, outs, ins)))


def gen_v0(M, nr):
    """(vr, vi) = V0' of output node 0 (the accumulation's start)."""
    L = block_layout(M)
    ps, pidx = pairs_of([L["v0re"], L["v0im"]])
    lines = ["v_mov_b64_dpp %%0, %%%d row_newbcast:%d %s" % (2 + pidx[L["v0re"] // 16], L["v0re"] % 16, DPP),
             "v_mov_b64_dpp %%1, %%%d row_newbcast:%d %s" % (2 + pidx[L["v0im"] // 16], L["v0im"] % 16, DPP)]
    outs = ['"=&v"(vr)', '"=&v"(vi)']
    ins = ['"v"(w[%d])' % p for p in ps]
    return ("template <> __device__ __forceinline__ void pf_v0<%d>(double& vr, double& vi, "
            "const double (&w)[%d]) {\n%s}\n" % (M, nr, asm_stmt(lines, outs, ins)))


def gen_bcast_group(name, M, groups, nr, extra_sig=""):
    """Outputs out_j[i] = entry groups[j] + i, i < M (early-clobber movs)."""
    ents = [g + i for g in groups for i in range(M)]
    ps, pidx = pairs_of(ents)
    n_out = len(groups) * M
    lines = []
    for j, g in enumerate(groups):
        for i in range(M):
            e = g + i
            lines.append("v_mov_b64_dpp %%%d, %%%d row_newbcast:%d %s"
                         % (j * M + i, n_out + pidx[e // 16], e % 16, DPP))
    outs = ['"=&v"(o%d[%d])' % (j, i) for j in range(len(groups)) for i in range(M)]
    ins = ['"v"(w[%d])' % p for p in ps]
    args = ", ".join("double (&o%d)[%d]" % (j, M) for j in range(len(groups)))
    return ("template <> __device__ __forceinline__ void %s<%d>(%s, const double (&w)[%d]) {\n%s}\n"
            % (name, M, args, nr, asm_stmt(lines, outs, ins)))


def gen_power(M, k, ns):
    """s_r = s0r[k] + pc fr[k] ; s_i = s0i[k] + qc fi[k]  (resident s tables, ns pairs)."""
    e_sr, e_si, e_fr, e_fi = k, M + k, 2 * M + k, 3 * M + k
    ps, pidx = pairs_of([e_sr, e_si, e_fr, e_fi])
    base = 2
    op = lambda e: "%%%d" % (base + pidx[e // 16])
    pc = "%%%d" % (base + len(ps))
    qc = "%%%d" % (base + len(ps) + 1)
    lines = ["v_mov_b64_dpp %%0, %s row_newbcast:%d %s" % (op(e_sr), e_sr % 16, DPP),
             "v_fmac_f64_dpp %%0, %s, %s row_newbcast:%d %s" % (op(e_fr), pc, e_fr % 16, DPP),
             "v_mov_b64_dpp %%1, %s row_newbcast:%d %s" % (op(e_si), e_si % 16, DPP),
             "v_fmac_f64_dpp %%1, %s, %s row_newbcast:%d %s" % (op(e_fi), qc, e_fi % 16, DPP)]
    outs = ['"=&v"(s_r)', '"=&v"(s_i)']
    ins = ['"v"(s[%d])' % p for p in ps] + ['"v"(pc)', '"v"(qc)']
    return ("template <> __device__ __forceinline__ void pf_power<%d, %d>(\n"
            "    double& s_r, double& s_i, const double (&s)[%d], double pc, double qc) {\n%s}\n"
            % (M, k, ns, asm_stmt(lines, outs, ins)))


def gen_od_elem(M, k):
    """The OpenDSS solve's per-element Yeq powers from its resident table y (2
    pairs: y0' re, y0' im; entry k in lane k % 16): y0r, y0i of element k."""
    lines = ["v_mov_b64_dpp %%%d, %%2 row_newbcast:%d %s" % (0, k % 16, DPP),
             "v_mov_b64_dpp %%%d, %%3 row_newbcast:%d %s" % (1, k % 16, DPP)]
    outs = ['"=&v"(y0r)', '"=&v"(y0i)']
    ins = ['"v"(y[0])', '"v"(y[1])']
    return ("template <> __device__ __forceinline__ void pf_od_elem<%d, %d>(\n"
            "    double& y0r, double& y0i, const double (&y)[2]) {\n%s}\n"
            % (M, k, asm_stmt(lines, outs, ins)))


def gen_bc16(k):
    """Entry k of a 16-entry resident pair (lane k % 16 of each row)."""
    lines = ["v_mov_b64_dpp %%0, %%1 row_newbcast:%d %s" % (k, DPP)]
    return ("template <> __device__ __forceinline__ double pf_bc16<%d>(double y) {\n  double r;\n%s  return r;\n}\n"
            % (k, asm_stmt(lines, ['"=&v"(r)'], ['"v"(y)'])))


def gen_band(M, k, nr):
    L = block_layout(M)
    es = [L["lo2"] + k, L["mn2"] + k, L["mx2"] + k]
    ps, pidx = pairs_of(es)
    lines = ["v_mov_b64_dpp %%%d, %%%d row_newbcast:%d %s" % (j, 3 + pidx[e // 16], e % 16, DPP)
             for j, e in enumerate(es)]
    outs = ['"=&v"(lo2)', '"=&v"(mn2)', '"=&v"(mx2)']
    ins = ['"v"(w[%d])' % p for p in ps]
    return ("template <> __device__ __forceinline__ void pf_band<%d, %d>(\n"
            "    double& lo2, double& mn2, double& mx2, const double (&w)[%d]) {\n%s}\n"
            % (M, k, nr, asm_stmt(lines, outs, ins)))


def gen_rows(M):
    """Output rows from resident row pairs (pf_rows_out): one row's operands --
    V0 re, im, then G re and G im of every element, slot j of the row in lane
    j % 16 of pair j // 16 -- fed by row_newbcast.  Four rows interleaved (eight
    independent FMA chains: one DPP wave per SIMD needs about eight to approach
    the fp64 issue rate, tools/micro/fp64_issue.hip), and a single row; per row the operations and their
    order are pf_node_pu's: vr = V0r, then per element fma(gr, ir), fma(-gi, ii)
    into vr and fma(gr, ii), fma(gi, ir) into vi."""
    npr = (2 * M + 2 + 15) // 16
    res = []
    for rows in (4, 1):
        names = "abcd"[:rows]
        w = lambda r, j: "%%%d" % (2 * rows + r * npr + j // 16)
        base = 2 * rows + rows * npr
        ir = lambda k: "%%%d" % (base + k)
        ii = lambda k: "%%%d" % (base + M + k)
        vr = lambda r: "%%%d" % (2 * r)
        vi = lambda r: "%%%d" % (2 * r + 1)
        lines = []
        for r in range(rows):
            lines += ["v_mov_b64_dpp %s, %s row_newbcast:0 %s" % (vr(r), w(r, 0), DPP),
                      "v_mov_b64_dpp %s, %s row_newbcast:1 %s" % (vi(r), w(r, 1), DPP)]
        # one wave per SIMD issues in order: a chain's next FMA sits 2 * rows
        # instructions behind its previous one (never back to back), so the
        # fp64 FMA latency overlaps the other chains' issue
        for k in range(M):
            gr, gi = 2 + k, 2 + M + k
            for r in range(rows):
                lines += ["v_fmac_f64_dpp %s, %s, %s row_newbcast:%d %s" % (vr(r), w(r, gr), ir(k), gr % 16, DPP),
                          "v_fmac_f64_dpp %s, %s, %s row_newbcast:%d %s" % (vi(r), w(r, gr), ii(k), gr % 16, DPP)]
            for r in range(rows):
                lines += ["v_fmac_f64_dpp %s, -%s, %s row_newbcast:%d %s" % (vr(r), w(r, gi), ii(k), gi % 16, DPP),
                          "v_fmac_f64_dpp %s, %s, %s row_newbcast:%d %s" % (vi(r), w(r, gi), ir(k), gi % 16, DPP)]
        outs = []
        for r in names:
            outs += ['"=&v"(%sr)' % r, '"=&v"(%si)' % r]
        ins = ['"v"(w%s[%d])' % (r, p) for r in names for p in range(npr)] + \
              ['"v"(ir[%d])' % k for k in range(M)] + ['"v"(ii[%d])' % k for k in range(M)]
        if rows == 4:
            sig = ("template <> __device__ __forceinline__ void pf_row4_dpp<%d>(\n"
                   "    double& ar, double& ai, double& br, double& bi, double& cr, double& ci,\n"
                   "    double& dr, double& di, const double (&wa)[%d], const double (&wb)[%d],\n"
                   "    const double (&wc)[%d], const double (&wd)[%d], const double (&ir)[%d],\n"
                   "    const double (&ii)[%d]) {\n" % (M, npr, npr, npr, npr, M, M))
        else:
            sig = ("template <> __device__ __forceinline__ void pf_row1_dpp<%d>(\n"
                   "    double& ar, double& ai, const double (&wa)[%d], const double (&ir)[%d],\n"
                   "    const double (&ii)[%d]) {\n" % (M, npr, M, M))
        res.append(sig + asm_stmt(lines, outs, ins) + "}\n")
    return "\n".join(res)


def main():
    ns = (4 * 16 + 15) // 16          # resident s tables: 4 x PGW_PF_MAX_M entries
    out = ["// GENERATED by gen_pf_dpp.py -- do not edit.  DPP-broadcast asm groups of",
           "// the power-flow solve (see gen_pf_dpp.py for the layout and hazard rule).",
           "template <int M, int K> __device__ __forceinline__ void pf_column(",
           "    double (&A)[M], double (&B)[M], double (&C)[M], const double (&w)[PFBlock<M>::kPairs],",
           "    double ir, double ii, double is);",
           "template <int M> __device__ __forceinline__ void pf_acc_init(",
           "    double (&o0)[M], double (&o1)[M], const double (&w)[PFBlock<M>::kPairs]);",
           "template <int M> __device__ __forceinline__ void pf_u0(",
           "    double (&o0)[M], double (&o1)[M], const double (&w)[PFBlock<M>::kPairs]);",
           "template <int M, int K> __device__ __forceinline__ void pf_power(",
           "    double& s_r, double& s_i, const double (&s)[kSPairs], double pc, double qc);",
           "template <int M, int K> __device__ __forceinline__ void pf_band(",
           "    double& lo2, double& mn2, double& mx2, const double (&w)[PFBlock<M>::kPairs]);",
           "template <int M> __device__ __forceinline__ void pf_node0(",
           "    double& vr, double& vi, const double (&w)[PFBlock<M>::kPairs], const double (&ir)[M],",
           "    const double (&ii)[M]);",
           "template <int M, int K> __device__ __forceinline__ void pf_column_v(",
           "    double (&A)[M], double (&B)[M], double (&C)[M], double& vr, double& vi,",
           "    const double (&w)[PFBlock<M>::kPairs], double ir, double ii, double is);",
           "template <int M> __device__ __forceinline__ void pf_v0(",
           "    double& vr, double& vi, const double (&w)[PFBlock<M>::kPairs]);",
           "template <int M> __device__ __forceinline__ void pf_row4_dpp(",
           "    double& ar, double& ai, double& br, double& bi, double& cr, double& ci, double& dr,",
           "    double& di, const double (&wa)[PFRow<M>::kPairs], const double (&wb)[PFRow<M>::kPairs],",
           "    const double (&wc)[PFRow<M>::kPairs], const double (&wd)[PFRow<M>::kPairs],",
           "    const double (&ir)[M], const double (&ii)[M]);",
           "template <int M, int K> __device__ __forceinline__ void pf_od_elem(",
           "    double& y0r, double& y0i, const double (&y)[2]);",
           "template <int K> __device__ __forceinline__ double pf_bc16(double y);",
           "template <int M> __device__ __forceinline__ void pf_row1_dpp(",
           "    double& ar, double& ai, const double (&wa)[PFRow<M>::kPairs], const double (&ir)[M],",
           "    const double (&ii)[M]);",
           ""]
    for k in range(16):
        out.append(gen_bc16(k))
    for M in SIZES:
        L = block_layout(M)
        nr = (L["size"] + 15) // 16
        out.append("// ---- M = %d (%d resident pairs)" % (M, nr))
        out.append(gen_bcast_group("pf_acc_init", M, [L["u0re"], L["u0sum"]], nr))
        out.append(gen_bcast_group("pf_u0", M, [L["u0re"], L["u0im"]], nr))
        out.append(gen_node0(M, nr))
        out.append(gen_v0(M, nr))
        out.append(gen_rows(M))
        for k in range(M):
            out.append(gen_column(M, k))
            out.append(gen_column_v(M, k))
            out.append(gen_power(M, k, ns))
            out.append(gen_band(M, k, nr))
            out.append(gen_od_elem(M, k))
    sys.stdout.write("\n".join(out))


if __name__ == "__main__":
    main()
