// Sanitizer driver for the host feeder builder (csrc/pgw_feeder.cpp, SURVEY
// section 5: "ASan/UBSan build of the host C++").  tests/test_cpu_sanitize.py
// compiles it together with pgw_feeder.cpp under -fsanitize=address,undefined,
// feeds it the element list of a feeder (dumped from the Python builder), and
// compares its outputs with the library's.
//
// stdin (binary): int32 n_elems, n_nodes, m, n_out; n_elems pgw_feeder_elem;
//                 int32 ep[m], eq[m], out_nodes[n_out]
// stdout (binary): Y, Z (2 n n doubles each), I, V0 (2 n each), W (2 m m),
//                  U0 (2 m), G (2 n_out m), V0_out (2 n_out)
// Then the argument checks run on malformed input (each must fail cleanly).
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "pgw.h"

namespace pgw {
static char g_msg[512];
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_msg, sizeof(g_msg), fmt, ap);
  va_end(ap);
}
}  // namespace pgw

template <class T>
static bool rd(T* p, size_t count) {
  return fread(p, sizeof(T), count, stdin) == count;
}

int main() {
  int32_t hdr[4];
  if (!rd(hdr, 4)) return 2;
  const int ne = hdr[0], n = hdr[1], m = hdr[2], no = hdr[3];
  std::vector<pgw_feeder_elem> els(ne);
  std::vector<int32_t> ep(m), eq(m), out(no);
  if (!rd(els.data(), ne) || !rd(ep.data(), m) || !rd(eq.data(), m) || (no && !rd(out.data(), no))) return 2;
  std::vector<double> Y(2 * n * n), Z(2 * n * n), I(2 * n), V0(2 * n);
  if (pgw_feeder_build(els.data(), ne, n, Y.data(), Z.data(), I.data(), V0.data()) != PGW_OK) {
    fprintf(stderr, "build failed: %s\n", pgw::g_msg);
    return 3;
  }
  std::vector<double> W(2 * m * m), U0(2 * m), G(2 * (no ? no : 1) * m), V0o(2 * (no ? no : 1));
  if (pgw_pf_reduce(n, Z.data(), V0.data(), m, ep.data(), eq.data(), no, out.data(), W.data(), U0.data(),
                    G.data(), V0o.data()) != PGW_OK) {
    fprintf(stderr, "reduce failed: %s\n", pgw::g_msg);
    return 3;
  }
  fwrite(Y.data(), 8, Y.size(), stdout);
  fwrite(Z.data(), 8, Z.size(), stdout);
  fwrite(I.data(), 8, I.size(), stdout);
  fwrite(V0.data(), 8, V0.size(), stdout);
  fwrite(W.data(), 8, W.size(), stdout);
  fwrite(U0.data(), 8, U0.size(), stdout);
  fwrite(G.data(), 8, 2 * no * m, stdout);
  fwrite(V0o.data(), 8, 2 * no, stdout);
  // malformed input: every call must return PGW_ERR_ARG with a message, and
  // touch nothing out of bounds
  int bad = 0;
  bad += pgw_feeder_build(els.data(), 0, n, Y.data(), Z.data(), I.data(), V0.data()) == PGW_OK;
  std::vector<pgw_feeder_elem> e2 = els;
  e2[0].nphases = 7;
  bad += pgw_feeder_build(e2.data(), ne, n, Y.data(), Z.data(), I.data(), V0.data()) == PGW_OK;
  e2 = els;
  e2[ne - 1].node1[0] = n + 5;
  bad += pgw_feeder_build(e2.data(), ne, n, Y.data(), Z.data(), I.data(), V0.data()) == PGW_OK;
  std::vector<int32_t> ep2 = ep;
  ep2[0] = n;
  bad += pgw_pf_reduce(n, Z.data(), V0.data(), m, ep2.data(), eq.data(), no, out.data(), W.data(),
                       U0.data(), G.data(), V0o.data()) == PGW_OK;
  if (no) {
    std::vector<int32_t> out2 = out;
    out2[no - 1] = -3;
    bad += pgw_pf_reduce(n, Z.data(), V0.data(), m, ep.data(), eq.data(), no, out2.data(), W.data(),
                         U0.data(), G.data(), V0o.data()) == PGW_OK;
  }
  if (bad) {
    fprintf(stderr, "%d malformed calls were accepted\n", bad);
    return 4;
  }
  return 0;
}
