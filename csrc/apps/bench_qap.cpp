// QAP solver benchmark. Parity: reference bin/bench_qap.cu (sizes 2..39 on random, matched and block-diagonal
// matrices; solve_catch for every size, exhaustive solve for sizes < 9).
#include <chrono>
#include <cstdio>
#include <random>

#include "stencil/rt/argparse.hpp"
#include "stencil/topo/qap.hpp"

int main(int argc, char **argv) {
  int maxN = 39;
  stencil::ArgParser p("QAP benchmark (reference bin/bench_qap.cu)");
  p.option(&maxN, "--max", "largest size");
  if (!p.parse(argc, argv)) return p.need_help() ? 0 : 1;
  std::mt19937 rng(0);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  std::printf("kind,n,solver,seconds,cost\n");
  for (int n = 2; n <= maxN; ++n) {
    for (int kind = 0; kind < 3; ++kind) {
      Mat2D<double> bw(n, n), comm(n, n);
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
          if (kind == 0) {
            bw.at(i, j) = 1 + 100 * u(rng);
            comm.at(i, j) = u(rng);
          } else if (kind == 1) { // matched: traffic mirrors bandwidth
            bw.at(i, j) = (i == j) ? 1000 : 1 + 10 * ((i ^ j) & 1);
            comm.at(i, j) = (i == j) ? 0 : ((i ^ j) & 1 ? 10 : 1);
          } else { // block diagonal (nodes of 4)
            bw.at(i, j) = (i / 4 == j / 4) ? 100 : 1;
            comm.at(i, j) = (i / 4 == j / 4) ? 0.1 : u(rng);
          }
        }
      const auto d = make_reciprocal(bw);
      const char *kinds[] = {"random", "matched", "blockdiag"};
      double c = 0;
      auto t0 = std::chrono::steady_clock::now();
      qap::solve_catch(comm, d, &c);
      std::printf("%s,%d,catch,%e,%e\n", kinds[kind], n,
                  std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(), c);
      if (n < 9) {
        t0 = std::chrono::steady_clock::now();
        qap::solve(comm, d, &c);
        std::printf("%s,%d,exact,%e,%e\n", kinds[kind], n,
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(), c);
      }
    }
  }
  return 0;
}
