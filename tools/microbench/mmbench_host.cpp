#include "host_linalg.hpp"
#include <chrono>
#include <cstdio>
#include <random>
using namespace pcamd;
int main() {
  std::mt19937_64 g(1); std::normal_distribution<double> nd;
  for (size_t n : {8, 64, 128, 256}) {
    Mat a(n, n), b(n, n);
    for (auto& v : a.a) v = nd(g) * 0.01;
    for (auto& v : b.a) v = nd(g);
    for (size_t i = 0; i < n; ++i) for (size_t j = i + 1; j < n; ++j) { a(j, i) = -a(i, j); }
    auto t0 = std::chrono::steady_clock::now();
    int reps = n <= 64 ? 200 : 20;
    Mat c;
    for (int r = 0; r < reps; ++r) c = matmul(a, b);
    auto t1 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) c = matrix_exp(a);
    auto t2 = std::chrono::steady_clock::now();
    double mm = std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
    double me = std::chrono::duration<double, std::micro>(t2 - t1).count() / reps;
    printf("n=%zu matmul %.1f us (%.1f GFLOP/s)  matrix_exp %.1f us  c00=%.17g\n", n, mm, 2.0*n*n*n/mm/1e3, me, c(0,0));
  }
}
