// Host-only check of csrc/transcript.h (no GPU needed): prints squeezes and
// Fr::random draws as canonical hex for comparison with hashlib / the oracle.
#include <cstdio>
#include "transcript.h"
using namespace h2g;
static void pr(const char* tag, const Fr& a) {
  const Fr c = to_canonical(a);
  printf("%s ", tag);
  for (int i = 7; i >= 0; i--) printf("%08x", c.l[i]);
  printf("\n");
}
int main() {
  uint8_t seed[32];
  for (int i = 0; i < 32; i++) seed[i] = 7;
  ChaChaRng rng(seed);
  for (int i = 0; i < 6; i++) pr("rand", rng.random_fr());
  std::vector<uint8_t> proof;
  Transcript tr(&proof);
  Fr x = from_u64<FrParams>(12345);
  tr.common_scalar(x);
  pr("sq", tr.squeeze());
  G1Affine g;
  g.x = Fq::one();
  g.y = from_u64<FqParams>(2);
  tr.write_point(g);
  pr("sq", tr.squeeze());
  pr("sq", tr.squeeze());
  tr.write_scalar(x);
  pr("sq", tr.squeeze());
  for (auto b : proof) printf("%02x", b);
  printf("\n");
}
