// CPU optimizers for the native TCP parameter server -- the same math and spec strings as
// ps_amd/parallel/updaters.py and the HIP kernels in csrc/kernels/optim.hip
// (reference: update/SimpleUpdater.java, AdamUpdater.java, FtrlUpdater.java).
#pragma once
#include <cmath>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace psnative {

inline bool spec_get(const std::string& spec, const std::string& key, double* out) {
  const std::string pat = key + ":";
  size_t pos = 0;
  while ((pos = spec.find(pat, pos)) != std::string::npos) {
    if (pos == 0 || spec[pos - 1] == '@') {
      size_t b = pos + pat.size();
      size_t e = spec.find('@', b);
      if (e == std::string::npos) return false;
      *out = std::strtod(spec.substr(b, e - b).c_str(), nullptr);
      return true;
    }
    pos += pat.size();
  }
  return false;
}

inline double spec_or(const std::string& spec, const std::string& key, double d) {
  double v;
  return spec_get(spec, key, &v) ? v : d;
}

// Per-key optimizer state lives with the key (Entry::states), the updater is stateless
// apart from its hyper-parameters; ``t`` is the key's step count (Adam bias correction).
class Updater {
 public:
  virtual ~Updater() = default;
  virtual int n_state() const = 0;
  virtual void update(float* w, const float* g, size_t n, std::vector<std::vector<float>>& st, long t) const = 0;
  std::string spec;
};

class SimpleUpdater : public Updater {
 public:
  explicit SimpleUpdater(const std::string& s) : eta(static_cast<float>(spec_or(s, "eta", 0.01))) { spec = s; }
  int n_state() const override { return 0; }
  void update(float* w, const float* g, size_t n, std::vector<std::vector<float>>&, long) const override {
    for (size_t i = 0; i < n; ++i) w[i] -= eta * g[i];
  }
  float eta;
};

class MomentumUpdater : public Updater {
 public:
  explicit MomentumUpdater(const std::string& s)
      : lr(spec_or(s, "lr", 0.1)), mom(spec_or(s, "momentum", 0.9)), wd(spec_or(s, "wd", 0.0)),
        nesterov(spec_or(s, "nesterov", 0.0) != 0.0) {
    spec = s;
  }
  int n_state() const override { return 1; }
  void update(float* w, const float* g, size_t n, std::vector<std::vector<float>>& st, long) const override {
    float* m = st[0].data();
    for (size_t i = 0; i < n; ++i) {
      float gi = g[i] + wd * w[i];
      m[i] = mom * m[i] + gi;
      w[i] -= lr * (nesterov ? gi + mom * m[i] : m[i]);
    }
  }
  float lr, mom, wd;
  bool nesterov;
};

class AdamUpdater : public Updater {
 public:
  explicit AdamUpdater(const std::string& s)
      : alfa(spec_or(s, "alfa", 0.001)), b1(spec_or(s, "beta1", 0.9)), b2(spec_or(s, "beta2", 0.999)),
        eps(spec_or(s, "epsilon", 1e-8)), bc(static_cast<int>(spec_or(s, "bc", 2))) {
    spec = s;
  }
  int n_state() const override { return 2; }
  void update(float* w, const float* g, size_t n, std::vector<std::vector<float>>& st, long t) const override {
    float c1 = 1.f, c2 = 1.f;
    if (bc == 2) {  // reference constant bias correction (AdamUpdater.java:63-64, Q5)
      c1 = 1.f / (1.f - b1);
      c2 = 1.f / (1.f - b2);
    } else if (bc == 1) {
      c1 = 1.f / (1.f - std::pow(b1, static_cast<float>(t)));
      c2 = 1.f / (1.f - std::pow(b2, static_cast<float>(t)));
    }
    float* m = st[0].data();
    float* v = st[1].data();
    for (size_t i = 0; i < n; ++i) {
      m[i] = b1 * m[i] + (1.f - b1) * g[i];
      v[i] = b2 * v[i] + (1.f - b2) * g[i] * g[i];
      w[i] -= alfa * (m[i] * c1) / (std::sqrt(v[i] * c2) + eps);
    }
  }
  float alfa, b1, b2, eps;
  int bc;
};

class AdagradUpdater : public Updater {
 public:
  explicit AdagradUpdater(const std::string& s)
      : lr(spec_or(s, "lr", 0.01)), eps(spec_or(s, "epsilon", 1e-10)), rowwise(spec_or(s, "rowwise", 0.0) != 0.0) {
    spec = s;
  }
  int n_state() const override { return 1; }
  void update(float* w, const float* g, size_t n, std::vector<std::vector<float>>& st, long) const override {
    float* h = st[0].data();
    if (rowwise) {  // one accumulator per key/row: h += mean(g^2) (the DLRM convention, optim.hip)
      float ss = 0.f;
      for (size_t i = 0; i < n; ++i) ss += g[i] * g[i];
      h[0] += n ? ss / static_cast<float>(n) : 0.f;
      const float denom = std::sqrt(h[0]) + eps;
      for (size_t i = 0; i < n; ++i) w[i] -= lr * g[i] / denom;
      return;
    }
    for (size_t i = 0; i < n; ++i) {
      h[i] += g[i] * g[i];
      w[i] -= lr * g[i] / (std::sqrt(h[i]) + eps);
    }
  }
  float lr, eps;
  bool rowwise;
};

// Philox-4x32-10, bit-identical to psamd::Philox (csrc/include/psamd_device.h) and
// ps_amd.ops.sparse.philox_u01: server-created rows get exactly the values the HIP lazy-init
// kernel gives the same (seed, key) on the GPU path.
// 128-bit counter (ctr low 64 bits, ctr_hi high 64 bits): lazily initialised rows use
// (element group, global key) so every key -- field bits included -- gets its own stream
inline float philox_u01(uint64_t seed, uint64_t ctr, int word = 0, uint64_t ctr_hi = 0) {
  uint32_t c[4] = {static_cast<uint32_t>(ctr), static_cast<uint32_t>(ctr >> 32), static_cast<uint32_t>(ctr_hi),
                   static_cast<uint32_t>(ctr_hi >> 32)};
  uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = static_cast<uint64_t>(0xD2511F53u) * c[0];
    const uint64_t p1 = static_cast<uint64_t>(0xCD9E8D57u) * c[2];
    const uint32_t hi0 = static_cast<uint32_t>(p0 >> 32), lo0 = static_cast<uint32_t>(p0);
    const uint32_t hi1 = static_cast<uint32_t>(p1 >> 32), lo1 = static_cast<uint32_t>(p1);
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return static_cast<float>(c[word & 3] >> 8) * (1.0f / 16777216.0f);
}

class FtrlUpdater : public Updater {
 public:
  explicit FtrlUpdater(const std::string& s, bool reference_mode)
      : alfa(spec_or(s, "alfa", 0.005)), beta(spec_or(s, "beta", 1.0)), l1(spec_or(s, "l1", 0.001)),
        l2(spec_or(s, "l2", 0.001)), ref(reference_mode) {
    spec = s;
  }
  int n_state() const override { return 2; }
  void update(float* w, const float* g, size_t n, std::vector<std::vector<float>>& st, long) const override {
    if (ref && n > 0 && g[0] == 0.f) return;  // FtrlUpdater.java:52-54
    float* z = st[0].data();
    float* nn = st[1].data();
    for (size_t i = 0; i < n; ++i) {
      const float gi = g[i];
      if (ref) {
        float wn = 0.f;
        if (std::fabs(z[i]) > l1) {
          const float sg = z[i] >= 0.f ? 1.f : -1.f;
          wn = -(z[i] - sg * l1) / ((l2 + (beta + std::sqrt(nn[i]))) / alfa);
        }
        const float sigma = std::sqrt(nn[i] + gi * gi) - std::sqrt(nn[i] / alfa);
        z[i] += gi - sigma * wn;
        nn[i] += gi * gi;
        w[i] = wn;
      } else {
        const float n2 = nn[i] + gi * gi;
        const float sigma = (std::sqrt(n2) - std::sqrt(nn[i])) / alfa;
        z[i] += gi - sigma * w[i];
        nn[i] = n2;
        if (std::fabs(z[i]) <= l1) w[i] = 0.f;
        else {
          const float sg = z[i] >= 0.f ? 1.f : -1.f;
          w[i] = -(z[i] - sg * l1) / ((beta + std::sqrt(n2)) / alfa + l2);
        }
      }
    }
  }
  float alfa, beta, l1, l2;
  bool ref;
};

inline std::unique_ptr<Updater> make_updater(const std::string& spec) {
  const std::string head = spec.substr(0, spec.find('@'));
  double tmp;
  if (head == "simple" || head == "sgd") return std::make_unique<SimpleUpdater>(spec);
  if (head == "momentum") return std::make_unique<MomentumUpdater>(spec);
  if (head == "adagrad") return std::make_unique<AdagradUpdater>(spec);
  if (head == "ftrl") return std::make_unique<FtrlUpdater>(spec, spec_or(spec, "reference", 0.0) != 0.0);
  if (head == "adam") {
    // the reference FtrlUpdater names itself "adam@alfa..@beta..@l1..@l2..@" (Q6)
    if (spec_get(spec, "l1", &tmp)) return std::make_unique<FtrlUpdater>(spec, true);
    return std::make_unique<AdamUpdater>(spec);
  }
  throw std::runtime_error("unknown updater spec: " + spec);
}

}  // namespace psnative
