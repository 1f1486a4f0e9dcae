// Random w_init stream of the reference (src/solver.rs:56-60, :112-118):
// rand 0.9 StdRng (ChaCha12Rng) seeded by SeedableRng::seed_from_u64 and
// rand_distr 0.5.1 StandardNormal (ZIGNOR ziggurat). Algorithms restated from
// the crates' published descriptions (a CPU restatement in the test
// infrastructure checks this file bit for bit).
#pragma once
#include <cstdint>

namespace pcamd {

class RustStdRng {
 public:
  explicit RustStdRng(uint64_t seed);  // StdRng::seed_from_u64
  uint32_t next_u32();
  uint64_t next_u64();                 // two keystream words, low first
  double standard_normal();            // rng.sample(StandardNormal) as f64

 private:
  void refill();
  uint32_t key_[8];
  uint64_t counter_ = 0;
  uint32_t buf_[16];
  int pos_ = 16;
};

}  // namespace pcamd
