// lattice_host.cpp — TEST ONLY: the product's lattice reduction (at2-node_amd/csrc/at2v_lattice.h)
// compiled for the host. Reads lines "k_hex s_hex" (little-endian 32-byte values as 64 hex digits,
// most significant first), prints "c0_hex c1_hex c1_neg bits t_hex" per line.
#include <cstdio>
#include <cstring>

#include "at2v_lattice.h"

using namespace at2v;

static bool parse(const char* h, uint32_t w[8]) {
  if (strlen(h) < 64) return false;
  for (int i = 0; i < 8; ++i) {
    unsigned v;
    if (sscanf(h + 8 * (7 - i), "%8x", &v) != 1) return false;
    w[i] = v;
  }
  return true;
}

static void put(const uint32_t w[8]) {
  for (int i = 7; i >= 0; --i) printf("%08x", w[i]);
}

int main() {
  char a[128], b[128];
  while (scanf("%127s %127s", a, b) == 2) {
    uint32_t k[8], s[8], t[8];
    if (!parse(a, k) || !parse(b, s)) return 2;
    HalfScalars h;
    lattice_reduce(h, k);
    sc_mul_signed(t, h, s);
    put(h.c0);
    printf(" ");
    put(h.c1);
    printf(" %d %d ", h.c1_neg, h.bits);
    put(t);
    printf("\n");
  }
  return 0;
}
