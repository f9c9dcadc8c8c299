// Writes a --distribution_file for `wals` (reference tool: qmf/gen_uniform.cpp:24-47):
// `count` values U(−bound, bound), one "%.9f" per line, to uniform.dat (or argv[3]).
// Seeded with argv[2] when given (the reference always uses random_device).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>

int main(int argc, char** argv) {
  const long long count = argc > 1 ? std::atoll(argv[1]) : 1000000;
  std::mt19937 gen(argc > 2 ? static_cast<unsigned>(std::atoll(argv[2])) : std::random_device()());
  const std::string out = argc > 3 ? argv[3] : "uniform.dat";
  std::uniform_real_distribution<double> distr(-0.01, 0.01);
  FILE* f = std::fopen(out.c_str(), "w");
  if (!f) {
    std::perror(out.c_str());
    return 1;
  }
  for (long long i = 0; i < count; ++i) std::fprintf(f, "%.9f\n", distr(gen));
  std::fclose(f);
  return 0;
}
