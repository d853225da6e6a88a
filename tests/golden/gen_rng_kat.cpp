// Generates RNG known answers from two independent implementations present in this image:
//  * torch's header-only at::philox_engine (ATen/core/PhiloxRNGEngine.h), which follows
//    curand's Philox4x32-10 layout (key = seed, counter.{z,w} = subsequence, 4 words/block);
//  * libstdc++'s std::mt19937_64 + uniform_int_distribution<uint64_t>(0, 2^64-1), exactly the
//    reference's launch-seed source (src/context/context.h:7-21).
// Output: JSON on stdout.  Built and run by tests/golden/make_golden.py.
#include <ATen/core/PhiloxRNGEngine.h>
#include <cstdio>
#include <random>
int main() {
  const unsigned long long cases[][3] = {
      {0ULL, 0ULL, 0ULL}, {123ULL, 0ULL, 0ULL}, {123ULL, 127ULL, 0ULL},
      {0xDEADBEEFCAFEBABEULL, 31ULL, 2ULL}, {42ULL * 1024ULL + 7ULL, 5ULL, 1ULL},
      {0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFULL, 3ULL}};
  printf("{\n \"philox\": [\n");
  const int n = sizeof(cases) / sizeof(cases[0]);
  for (int c = 0; c < n; ++c) {
    at::Philox4_32 eng(cases[c][0], cases[c][1], cases[c][2]);  // offset in 128-bit blocks
    printf("  {\"seed\": %llu, \"subsequence\": %llu, \"offset_words\": %llu, \"out\": [",
           cases[c][0], cases[c][1], cases[c][2] * 4ULL);
    for (int i = 0; i < 16; ++i) printf("%u%s", eng(), i < 15 ? ", " : "");
    printf("]}%s\n", c < n - 1 ? "," : "");
  }
  printf(" ],\n \"mt19937_64\": [\n");
  const unsigned long long seeds[] = {5489ULL, 0ULL, 20261015ULL};
  for (int s = 0; s < 3; ++s) {
    std::mt19937_64 gen(seeds[s]);
    std::uniform_int_distribution<unsigned long long> dis(0, 0xFFFFFFFFFFFFFFFFULL);
    printf("  {\"seed\": %llu, \"out\": [", seeds[s]);
    for (int i = 0; i < 8; ++i) printf("\"%llu\"%s", dis(gen), i < 7 ? ", " : "");
    printf("]}%s\n", s < 2 ? "," : "");
  }
  printf(" ]\n}\n");
  return 0;
}
