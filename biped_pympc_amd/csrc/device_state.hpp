// device_state.hpp -- per-device host state of libsrbd_mpc.so (one process may drive several GPUs).
//
// What the library remembers between calls is keyed by the HIP device current at the call:
// the dynamic-LDS attribute already configured for each kernel (hipFuncSetAttribute acts on the
// current device), the event pair of the CusADi-ABI blocking calls, and the solver-path selector.
// Host-only code with no HIP dependency, so tests/test_device_state.py compiles it with g++ and
// checks the keying on the CPU.
#pragma once
#include <cstddef>
#include <mutex>

namespace srbd {

constexpr int kMaxDevices = 64;

template <class T>
class PerDevice {
 public:
  // nullptr for a device index outside [0, kMaxDevices)
  T* at(int dev) { return (dev >= 0 && dev < kMaxDevices) ? &v_[dev] : nullptr; }
  const T* at(int dev) const { return (dev >= 0 && dev < kMaxDevices) ? &v_[dev] : nullptr; }

 private:
  T v_[kMaxDevices]{};
};

// Largest dynamic-LDS size configured for one kernel, per device. claim() returns true when the
// caller must (re)configure the attribute for `bytes` on `dev`; commit() records that it did.
class LdsAttr {
 public:
  bool claim(int dev, size_t bytes) {
    std::lock_guard<std::mutex> lock(mu_);
    const size_t* c = cfg_.at(dev);
    return c && bytes > *c;
  }
  void commit(int dev, size_t bytes) {
    std::lock_guard<std::mutex> lock(mu_);
    if (size_t* c = cfg_.at(dev))
      if (bytes > *c) *c = bytes;
  }
  size_t configured(int dev) const {
    const size_t* c = cfg_.at(dev);
    return c ? *c : 0;
  }

 private:
  std::mutex mu_;
  PerDevice<size_t> cfg_;
};

}  // namespace srbd
