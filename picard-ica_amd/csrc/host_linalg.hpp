// Host-side N×N linear algebra for the Picard driver (N ≤ a few hundred).
// Restates src/math.rs and the LAPACK calls the reference delegates to
// ndarray-linalg 0.18 (eigh → Jacobi, sln_det → partially pivoted LU).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace pcamd {

// Row-major dense matrix.
struct Mat {
  size_t rows = 0, cols = 0;
  std::vector<double> a;
  Mat() = default;
  Mat(size_t r, size_t c, double v = 0.0) : rows(r), cols(c), a(r * c, v) {}
  double& operator()(size_t i, size_t j) { return a[i * cols + j]; }
  double operator()(size_t i, size_t j) const { return a[i * cols + j]; }
  double* data() { return a.data(); }
  const double* data() const { return a.data(); }
  static Mat eye(size_t n) {
    Mat m(n, n);
    for (size_t i = 0; i < n; ++i) m(i, i) = 1.0;
    return m;
  }
};

Mat matmul(const Mat& a, const Mat& b);          // a·b
Mat matmul_nt(const Mat& a, const Mat& b);       // a·bᵀ
Mat transpose(const Mat& a);
Mat add(const Mat& a, const Mat& b);
Mat sub(const Mat& a, const Mat& b);
Mat scale(const Mat& a, double s);
double max_abs(const Mat& a);
// int8 digit image of W rows for the device Y stage (host_linalg.cpp)
// image [row block][digit][k-step < ksw][lane][16 B] (ksw = 2 for nf ≤ 128, 4 for nf ≤ 256)
void oz_split_rows(const double* w, size_t nc, size_t nf, uint8_t* img, double* sc, int ksw, double* dn2 = nullptr);
double dot_sum(const Mat& a, const Mat& b);       // Σ a∘b

// Symmetric eigendecomposition (cyclic Jacobi). Eigenvalues ascending (as
// LAPACK dsyev), eigenvectors in the columns of vecs.
void eigh(const Mat& s, std::vector<double>* vals, Mat* vecs);

// math.rs:12-33. Returns false on min eigenvalue < 1e-10 (SingularMatrix).
bool sym_decorrelation(const Mat& w, Mat* out);
// math.rs:38-74 Taylor + scaling & squaring.
Mat matrix_exp(const Mat& a);
// math.rs:84-88: (sign, log|det|), sign 0 and -inf for a singular matrix.
void sln_det(const Mat& m, double* sign, double* logabs);
// math.rs:91-93
Mat skew_symmetric(const Mat& a);
// JADE sweep kernels: a ← c·a − s·b, b ← s·a + c·b elementwise; and the
// g-sums of jade.rs:137-167 (Σ h_pq², Σ h_pq·h_d, Σ h_d², h_pq = 2·apq, h_d = app − aqq)
void givens_rows(double* a, double* b, size_t len, double c, double s);
void jade_gsums(const double* apq, const double* app, const double* aqq, size_t len, double* g);
// result.rs:68-129 Gauss-Jordan; false when a pivot < 1e-15.
bool invert_matrix(const Mat& m, Mat* out);

}  // namespace pcamd
