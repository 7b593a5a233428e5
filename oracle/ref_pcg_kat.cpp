// Known-answer generator compiled against the reference's vendored pcg header
// (/root/reference/external/pcg-cpp/include/pcg/pcg_random.hpp): pcg32_fast seeded with a
// given 64-bit value (RandomNumberGenerator::begin_job seeds with hash(seed, jid),
// include/vpt/random.hpp:93-95).  Usage: pcg32_fast_kat <seed64-hex> <n>  -> n u32 lines.
#include <cstdio>
#include <cstdlib>
#include <pcg/pcg_random.hpp>
int main(int argc, char** argv) {
  if (argc != 3) return 2;
  unsigned long long s = std::strtoull(argv[1], nullptr, 16);
  int n = std::atoi(argv[2]);
  pcg32_fast e;
  e.seed(s);
  for (int i = 0; i < n; ++i) std::printf("%u\n", (unsigned)e());
  return 0;
}
