// Host-side feeder model build (C++, no GPU): the native stand-in for the
// OpenDSS circuit build the reference triggers at opendss.py:36-51
// ("Redirect IEEE13Nodeckt.dss").  Assembles the 3-phase nodal admittance
// matrix of lines, 2-winding transformers and the Thevenin source (loads are
// NOT stamped: the batched solver treats them as current injections), inverts
// it, and reduces it onto the load elements for the device kernels.
//
// Element models follow OpenDSS's documented ones:
//   Vsource  |Z1| = kV^2/MVAsc3, X1/R1 given;  |2 Z1 + Z0| = 3 kV^2/MVAsc1 with
//            X0/R0 given (quadratic in R0);  Zs = (2Z1+Z0)/3, Zm = (Z0-Z1)/3;
//            Norton  Y = Zs^-1, I = Y E,  E = pu kV/sqrt3 at angle, -120, +120.
//   Transformer (2 windings, no magnetising branch): Zsc = (%r1+%r2)/100 + j XHL/100
//            on the kVA base, winding voltages kV/sqrt3 (3-phase wye) or kV
//            (delta); per phase  Yw = y [[1, -t], [-t, t^2]], t = Vw1/Vw2;
//            delta windings span phase p -> p+1.
//            Taps scale the winding voltages: t = (Vw1 tap1)/(Vw2 tap2), and the
//            leakage impedance is referred to winding 1 at Vw1 tap1.
//   Transformer, N windings (PGW_ELEM_XFMR_N, 2 or 3): OpenDSS's ZB form, see
//            pgw.h; explicit hi / lo terminal per winding and phase.
//   Line     Z = (R + jX) len,  Yc = j 2 pi f C 1e-9 len, split half/half.
//   Shunt    a constant admittance per phase (capacitor, constant-Z load).
#include <cmath>
#include <complex>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>

#include "pgw.h"

namespace pgw {
void set_error(const char* fmt, ...);
}

namespace {

using cplx = std::complex<double>;
using Mat = std::vector<cplx>;   // row-major square
using xcplx = std::complex<long double>;   // x87 80-bit: 64-bit mantissa
using XMat = std::vector<xcplx>;

// Gauss-Jordan inversion with partial pivoting; returns false if singular.
// Templated so the feeder matrix is inverted in extended precision: the
// near-ideal switch (1e-7 ohm) gives Y a condition number ~1e7, and an fp64
// inverse would carry ~1e-9 relative error into every load-element voltage.
template <typename CT>
bool invert(std::vector<CT>& a, int n) {
  using R = typename CT::value_type;
  std::vector<CT> inv(static_cast<size_t>(n) * n, CT(0, 0));
  for (int i = 0; i < n; ++i) inv[i * n + i] = R(1);
  for (int c = 0; c < n; ++c) {
    int piv = c;
    R best = std::abs(a[c * n + c]);
    for (int r = c + 1; r < n; ++r) {
      R v = std::abs(a[r * n + c]);
      if (v > best) {
        best = v;
        piv = r;
      }
    }
    if (best == R(0) || !std::isfinite(best)) return false;
    if (piv != c) {
      for (int j = 0; j < n; ++j) {
        std::swap(a[c * n + j], a[piv * n + j]);
        std::swap(inv[c * n + j], inv[piv * n + j]);
      }
    }
    CT d = R(1) / a[c * n + c];
    for (int j = 0; j < n; ++j) {
      a[c * n + j] *= d;
      inv[c * n + j] *= d;
    }
    for (int r = 0; r < n; ++r) {
      if (r == c) continue;
      CT f = a[r * n + c];
      if (f == CT(0, 0)) continue;
      for (int j = 0; j < n; ++j) {
        a[r * n + j] -= f * a[c * n + j];
        inv[r * n + j] -= f * inv[c * n + j];
      }
    }
  }
  a.swap(inv);
  return true;
}

struct Builder {
  int n;
  Mat Y;
  std::vector<cplx> I;
  explicit Builder(int nn) : n(nn), Y(static_cast<size_t>(nn) * nn), I(nn) {}

  // Y[nodes, nodes] += yp  (yp is k x k, nodes may contain -1 = ground)
  bool stamp(const std::vector<int>& nodes, const Mat& yp) {
    int k = static_cast<int>(nodes.size());
    for (int a = 0; a < k; ++a) {
      if (nodes[a] >= n) return false;
      if (nodes[a] < 0) continue;
      for (int b = 0; b < k; ++b) {
        if (nodes[b] < 0) continue;
        Y[nodes[a] * n + nodes[b]] += yp[a * k + b];
      }
    }
    return true;
  }
};

bool add_vsource(Builder& B, const pgw_feeder_elem& e) {
  const double kv = e.basekv;
  const double z1mag = kv * kv / e.mvasc3;
  const double x1 = z1mag * e.x1r1 / std::sqrt(1.0 + e.x1r1 * e.x1r1);
  const double r1 = x1 / e.x1r1;
  const double zs = 3.0 * kv * kv / e.mvasc1;   // |2 Z1 + Z0|
  const double qa = 1.0 + e.x0r0 * e.x0r0;
  const double qb = 4.0 * (r1 + x1 * e.x0r0);
  const double qc = 4.0 * (r1 * r1 + x1 * x1) - zs * zs;
  const double r0 = (-qb + std::sqrt(qb * qb - 4.0 * qa * qc)) / (2.0 * qa);
  const double x0 = r0 * e.x0r0;
  const cplx Z1(r1, x1), Z0(r0, x0);
  const cplx zself = (2.0 * Z1 + Z0) / 3.0, zmut = (Z0 - Z1) / 3.0;
  Mat Zs(9);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Zs[i * 3 + j] = (i == j) ? zself : zmut;
  if (!invert(Zs, 3)) return false;
  const double vln = e.pu * kv * 1000.0 / std::sqrt(3.0);
  const double deg = M_PI / 180.0;
  cplx E[3];
  const double ang[3] = {0.0, -120.0, 120.0};
  for (int p = 0; p < 3; ++p) E[p] = std::polar(vln, (e.angle + ang[p]) * deg);
  std::vector<int> nodes(e.node1, e.node1 + 3);
  if (!B.stamp(nodes, Zs)) return false;
  for (int a = 0; a < 3; ++a) {
    cplx s(0.0, 0.0);
    for (int b = 0; b < 3; ++b) s += Zs[a * 3 + b] * E[b];
    if (nodes[a] >= 0) B.I[nodes[a]] += s;
  }
  return true;
}

bool add_transformer(Builder& B, const pgw_feeder_elem& e) {
  const int ph = e.nphases;
  const double s3 = std::sqrt(3.0);
  const double vw1 = e.kv1 * 1000.0 / ((e.conn1 == 0 && ph == 3) ? s3 : 1.0);
  const double vw2 = e.kv2 * 1000.0 / ((e.conn2 == 0 && ph == 3) ? s3 : 1.0);
  const double kva_ph = e.kva * 1000.0 / ph;
  const double v1 = vw1 * (e.tap1 != 0.0 ? e.tap1 : 1.0), v2 = vw2 * (e.tap2 != 0.0 ? e.tap2 : 1.0);
  const cplx zpu((e.pct_r1 + e.pct_r2) / 100.0, e.xhl / 100.0);
  const cplx y = 1.0 / (zpu * (v1 * v1 / kva_ph));
  const double t = v1 / v2;
  const cplx yw[4] = {y, -t * y, -t * y, t * t * y};
  for (int p = 0; p < ph; ++p) {
    // terminal list: [w1 hi, w1 lo, w2 hi, w2 lo]; winding voltage = hi - lo
    std::vector<int> nodes = {e.node1[p], e.conn1 ? e.node1[(p + 1) % ph] : -1, e.node2[p],
                              e.conn2 ? e.node2[(p + 1) % ph] : -1};
    const double sgn[4] = {1.0, -1.0, 1.0, -1.0};
    const int w_of[4] = {0, 0, 1, 1};
    Mat yp(16);
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b) yp[a * 4 + b] = sgn[a] * sgn[b] * yw[w_of[a] * 2 + w_of[b]];
    if (!B.stamp(nodes, yp)) return false;
  }
  return true;
}

// PGW_ELEM_XFMR_N (pgw.h): OpenDSS's N-winding leakage model, explicit terminals.
bool add_transformer_n(Builder& B, const pgw_feeder_elem& e) {
  const int ph = e.nphases, nw = e.nwindings;
  if (nw < 2 || nw > 3) return false;
  const double s3 = std::sqrt(3.0);
  const double kv[3] = {e.kv1, e.kv2, e.kv3}, tap[3] = {e.tap1, e.tap2, e.tap3};
  const double kva[3] = {e.kva, e.kva2 > 0.0 ? e.kva2 : e.kva, e.kva3 > 0.0 ? e.kva3 : e.kva};
  const double pct_r[3] = {e.pct_r1, e.pct_r2, e.pct_r3};
  const int conn[3] = {e.conn1, e.conn2, e.conn3};
  double v[3], r[3];
  for (int k = 0; k < nw; ++k) {
    v[k] = kv[k] * 1000.0 / ((conn[k] == 0 && ph == 3) ? s3 : 1.0) * (tap[k] != 0.0 ? tap[k] : 1.0);
    r[k] = pct_r[k] / 100.0 * (kva[0] / kva[k]);     // on winding 1's kVA
  }
  // ZB: winding k+1 against winding 1 (pu on winding 1's kVA)
  const cplx z12(r[0] + r[1], e.xhl / 100.0);
  Mat ZB;
  if (nw == 2) {
    ZB = {z12};
  } else {
    const cplx z13(r[0] + r[2], e.xht / 100.0), z23(r[1] + r[2], e.xlt / 100.0);
    const cplx zm = 0.5 * (z12 + z13 - z23);
    ZB = {z12, zm, zm, z13};
  }
  if (!invert(ZB, nw - 1)) return false;
  // Y_pu = A ZB^-1 A^T: row / column 0 = -(sums), the rest ZB^-1
  Mat Yw(static_cast<size_t>(nw) * nw);
  const int q = nw - 1;
  cplx tot(0.0, 0.0);
  for (int i = 0; i < q; ++i) {
    cplx row(0.0, 0.0);
    for (int j = 0; j < q; ++j) {
      Yw[(i + 1) * nw + (j + 1)] = ZB[i * q + j];
      row += ZB[i * q + j];
    }
    Yw[(i + 1) * nw] = -row;
    Yw[i + 1] = -row;                                 // (ZB^-1 symmetric)
    tot += row;
  }
  Yw[0] = tot;
  const double s_ph = kva[0] * 1000.0 / ph;
  for (int i = 0; i < nw; ++i)
    for (int j = 0; j < nw; ++j) Yw[i * nw + j] *= s_ph / (v[i] * v[j]);
  for (int p = 0; p < ph; ++p) {
    std::vector<int> nodes;
    for (int k = 0; k < nw; ++k) {
      nodes.push_back(e.wnode[(k * 3 + p) * 2]);
      nodes.push_back(e.wnode[(k * 3 + p) * 2 + 1]);
    }
    const int nt = 2 * nw;
    Mat yp(static_cast<size_t>(nt) * nt);
    for (int a = 0; a < nt; ++a)
      for (int b = 0; b < nt; ++b)
        yp[a * nt + b] = ((a & 1) ? -1.0 : 1.0) * ((b & 1) ? -1.0 : 1.0) * Yw[(a >> 1) * nw + (b >> 1)];
    if (!B.stamp(nodes, yp)) return false;
  }
  return true;
}

bool add_line(Builder& B, const pgw_feeder_elem& e) {
  const int ph = e.nphases;
  Mat Z(static_cast<size_t>(ph) * ph);
  Mat Yc(static_cast<size_t>(ph) * ph);
  const double w = 2.0 * M_PI * e.freq;
  for (int i = 0; i < ph; ++i)
    for (int j = 0; j < ph; ++j) {
      Z[i * ph + j] = cplx(e.r[i * ph + j], e.x[i * ph + j]) * e.length;
      Yc[i * ph + j] = cplx(0.0, w * e.c[i * ph + j] * 1e-9 * e.length);
    }
  if (!invert(Z, ph)) return false;
  const int k = 2 * ph;
  Mat yp(static_cast<size_t>(k) * k);
  for (int i = 0; i < ph; ++i)
    for (int j = 0; j < ph; ++j) {
      const cplx ys = Z[i * ph + j], half = 0.5 * Yc[i * ph + j];
      yp[i * k + j] = ys + half;
      yp[(i + ph) * k + (j + ph)] = ys + half;
      yp[i * k + (j + ph)] = -ys;
      yp[(i + ph) * k + j] = -ys;
    }
  std::vector<int> nodes;
  for (int p = 0; p < ph; ++p) nodes.push_back(e.node1[p]);
  for (int p = 0; p < ph; ++p) nodes.push_back(e.node2[p]);
  return B.stamp(nodes, yp);
}

bool add_shunt(Builder& B, const pgw_feeder_elem& e) {
  for (int p = 0; p < e.nphases; ++p) {
    const cplx y(e.r[p], e.x[p]);
    const Mat yp = {y, -y, -y, y};
    if (!B.stamp({e.node1[p], e.node2[p]}, yp)) return false;
  }
  return true;
}

void put(double* dst, const cplx* src, size_t count) {
  for (size_t i = 0; i < count; ++i) {
    dst[2 * i] = src[i].real();
    dst[2 * i + 1] = src[i].imag();
  }
}

}  // namespace

extern "C" {

int32_t pgw_struct_sizes(int64_t* out, int32_t n) {
  const int64_t sz[PGW_N_STRUCT_SIZES] = {
      (int64_t)sizeof(pgw_mat),           (int64_t)sizeof(pgw_battery_params),
      (int64_t)sizeof(pgw_pv_params),     (int64_t)sizeof(pgw_building_params),
      (int64_t)sizeof(pgw_building_exo),  (int64_t)sizeof(pgw_building_ext),
      (int64_t)sizeof(pgw_ev_params),     (int64_t)sizeof(pgw_ev_step_info),
      (int64_t)sizeof(pgw_reduce_args),   (int64_t)sizeof(pgw_pf_params),
      (int64_t)sizeof(pgw_pf_tables),     (int64_t)sizeof(pgw_feeder_elem),
      (int64_t)sizeof(pgw_coord_params),  (int64_t)sizeof(pgw_coord_buffers),
      (int64_t)sizeof(pgw_coord_step_info), (int64_t)sizeof(pgw_pred_meta),
      (int64_t)sizeof(pgw_hs_params),       (int64_t)sizeof(pgw_hs_step_info),
      (int64_t)sizeof(pgw_hs_buffers),      (int64_t)sizeof(pgw_mc_step_args),
      (int64_t)sizeof(pgw_matf),            (int64_t)sizeof(pgw_coord_buffers_f32),
      (int64_t)sizeof(pgw_ma_step_args),   (int64_t)sizeof(pgw_pfg_elem),
      (int64_t)sizeof(pgw_pfg_params),     (int64_t)sizeof(pgw_pfg_tables),
      (int64_t)sizeof(pgw_reg_params),    (int64_t)sizeof(pgw_mc_step_dyn),
      (int64_t)sizeof(pgw_pf_od),         (int64_t)sizeof(pgw_mc_step_args_f32)};
  for (int i = 0; i < n && i < PGW_N_STRUCT_SIZES; ++i) out[i] = sz[i];
  return PGW_N_STRUCT_SIZES;
}

int32_t pgw_feeder_build(const pgw_feeder_elem* elems, int32_t n_elems, int32_t n_nodes, double* Y,
                         double* Z, double* I_src, double* V0) {
  if (!elems || n_elems <= 0 || n_nodes <= 0) {
    pgw::set_error("pgw_feeder_build: empty feeder");
    return PGW_ERR_ARG;
  }
  try {
    Builder B(n_nodes);
    for (int i = 0; i < n_elems; ++i) {
      const pgw_feeder_elem& e = elems[i];
      if (e.nphases < 1 || e.nphases > 3) {
        pgw::set_error("pgw_feeder_build: element %d has %d phases", i, e.nphases);
        return PGW_ERR_ARG;
      }
      bool ok = false;
      switch (e.kind) {
        case PGW_ELEM_VSOURCE: ok = add_vsource(B, e); break;
        case PGW_ELEM_XFMR: ok = add_transformer(B, e); break;
        case PGW_ELEM_XFMR_N: ok = add_transformer_n(B, e); break;
        case PGW_ELEM_LINE: ok = add_line(B, e); break;
        case PGW_ELEM_SHUNT: ok = add_shunt(B, e); break;
        default: ok = false;
      }
      if (!ok) {
        pgw::set_error("pgw_feeder_build: element %d (kind %d) is invalid", i, e.kind);
        return PGW_ERR_ARG;
      }
    }
    if (Y) put(Y, B.Y.data(), B.Y.size());
    if (I_src) put(I_src, B.I.data(), B.I.size());
    XMat Zx(B.Y.size());
    for (size_t i = 0; i < B.Y.size(); ++i) Zx[i] = xcplx(B.Y[i].real(), B.Y[i].imag());
    if (!invert(Zx, n_nodes)) {
      pgw::set_error("pgw_feeder_build: singular admittance matrix (floating node?)");
      return PGW_ERR_ARG;
    }
    Mat Zm(Zx.size());
    for (size_t i = 0; i < Zx.size(); ++i)
      Zm[i] = cplx((double)Zx[i].real(), (double)Zx[i].imag());
    if (Z) put(Z, Zm.data(), Zm.size());
    if (V0) {
      std::vector<cplx> v(n_nodes);
      for (int r = 0; r < n_nodes; ++r) {
        xcplx s(0, 0);
        for (int c = 0; c < n_nodes; ++c)
          s += Zx[r * n_nodes + c] * xcplx(B.I[c].real(), B.I[c].imag());
        v[r] = cplx((double)s.real(), (double)s.imag());
      }
      put(V0, v.data(), v.size());
    }
  } catch (...) {
    pgw::set_error("pgw_feeder_build: allocation failure");
    return PGW_ERR_ARG;
  }
  return PGW_OK;
}

int32_t pgw_pf_reduce(int32_t n, const double* Zi, const double* V0i, int32_t m, const int32_t* ep,
                      const int32_t* eq, int32_t n_out, const int32_t* out_nodes, double* W,
                      double* U0, double* G, double* V0_out) {
  if (!Zi || !V0i || !ep || !eq || m <= 0 || n <= 0 || (n_out > 0 && !out_nodes)) {
    pgw::set_error("pgw_pf_reduce: null argument");
    return PGW_ERR_ARG;
  }
  for (int k = 0; k < m; ++k)
    if (ep[k] < 0 || ep[k] >= n || eq[k] >= n) {
      pgw::set_error("pgw_pf_reduce: element %d node out of range", k);
      return PGW_ERR_ARG;
    }
  auto z = [&](int r, int c) { return cplx(Zi[2 * (r * n + c)], Zi[2 * (r * n + c) + 1]); };
  auto v0 = [&](int r) { return cplx(V0i[2 * r], V0i[2 * r + 1]); };
  // ZC[r][k] = (Z C^T)[r][k] = Z[r][p_k] - Z[r][q_k]
  std::vector<cplx> ZC(static_cast<size_t>(n) * m);
  for (int r = 0; r < n; ++r)
    for (int k = 0; k < m; ++k) {
      cplx s = z(r, ep[k]);
      if (eq[k] >= 0) s -= z(r, eq[k]);
      ZC[r * m + k] = s;
    }
  if (W) {
    for (int i = 0; i < m; ++i)
      for (int k = 0; k < m; ++k) {
        cplx s = ZC[ep[i] * m + k];
        if (eq[i] >= 0) s -= ZC[eq[i] * m + k];
        s = -s;
        W[2 * (i * m + k)] = s.real();
        W[2 * (i * m + k) + 1] = s.imag();
      }
  }
  if (U0) {
    for (int i = 0; i < m; ++i) {
      cplx s = v0(ep[i]);
      if (eq[i] >= 0) s -= v0(eq[i]);
      U0[2 * i] = s.real();
      U0[2 * i + 1] = s.imag();
    }
  }
  for (int o = 0; o < n_out; ++o) {
    int r = out_nodes[o];
    if (r < 0 || r >= n) {
      pgw::set_error("pgw_pf_reduce: output node %d out of range", r);
      return PGW_ERR_ARG;
    }
    if (G)
      for (int k = 0; k < m; ++k) {
        cplx s = -ZC[r * m + k];
        G[2 * (o * m + k)] = s.real();
        G[2 * (o * m + k) + 1] = s.imag();
      }
    if (V0_out) {
      V0_out[2 * o] = v0(r).real();
      V0_out[2 * o + 1] = v0(r).imag();
    }
  }
  return PGW_OK;
}

}  // extern "C"
