// Host N×N cost on the critical path of an orthogonal iteration: matmul and
// matrix_exp (math.rs:38-74 order) at N = 128, as host_solver.cpp calls them.
// Build: g++ -O3 -std=c++17 -fopenmp -I../../picard-ica_amd/csrc -I../../include expm_host.cpp
//        ../../picard-ica_amd/build/host_linalg.o -o expm_host
#include "host_linalg.hpp"
#include <chrono>
#include <cstdio>
#include <random>
using namespace pcamd;
static double now() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int main() {
  const size_t n = 128;
  std::mt19937_64 g(1);
  std::normal_distribution<double> nd(0, 1);
  for (double scale : {0.005, 0.02, 0.1}) {
    Mat a(n, n), w(n, n);
    for (auto& v : a.a) v = nd(g) * scale;
    for (size_t i = 0; i < n; ++i)
      for (size_t j = 0; j <= i; ++j) a(i, j) = i == j ? 0.0 : -a(j, i);
    for (auto& v : w.a) v = nd(g);
    double tm = 1e9, te = 1e9;
    for (int rep = 0; rep < 20; ++rep) {
      const double t0 = now();
      Mat m = matmul(a, w);
      const double t1 = now();
      Mat e = matmul(matrix_exp(a), w);
      const double t2 = now();
      if (t1 - t0 < tm) tm = t1 - t0;
      if (t2 - t1 < te) te = t2 - t1;
    }
    std::printf("max|D| %.3f: matmul %.3f ms, expm(D)*W %.3f ms (best of 20)\n", max_abs(a), tm, te);
  }
}
