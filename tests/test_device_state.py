"""Per-device host state of libsrbd_mpc.so (csrc/device_state.hpp) on the CPU: the header has no
HIP dependency, so it is compiled with g++ into a small driver that exercises the keying a process
driving several GPUs relies on: configured LDS limits, event slots and the
solver path are independent per device index, and out-of-range indices are refused."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = r"""
#include <cstdio>
#include "device_state.hpp"
int main() {
  using namespace srbd;
  int fails = 0;
  auto check = [&](bool c, const char* what) { if (!c) { std::printf("FAIL %s\n", what); ++fails; } };
  LdsAttr a;
  check(a.claim(0, 1024), "fresh device 0 needs configuring");
  a.commit(0, 1024);
  check(!a.claim(0, 1024) && !a.claim(0, 512), "device 0 configured for <= 1024");
  check(a.claim(0, 4096), "a larger request re-configures");
  check(a.claim(3, 512), "device 3 is independent of device 0");
  a.commit(3, 512);
  check(a.configured(0) == 1024 && a.configured(3) == 512 && a.configured(1) == 0, "per-device values");
  a.commit(3, 256);
  check(a.configured(3) == 512, "commit never lowers the configured size");
  check(!a.claim(-1, 8) && !a.claim(kMaxDevices, 8), "out-of-range devices are refused");
  PerDevice<int> path;
  *path.at(2) = 1;
  check(*path.at(2) == 1 && *path.at(0) == 0 && *path.at(63) == 0, "solver path per device");
  check(path.at(64) == nullptr && path.at(-1) == nullptr, "no slot outside [0, 64)");
  struct Ev { void* e[2]; };
  PerDevice<Ev> ev;
  check(ev.at(5)->e[0] == nullptr && ev.at(5)->e[1] == nullptr, "event slots start empty");
  std::printf("%d\n", fails);
  return fails;
}
"""


def test_device_keyed_host_state(tmp_path):
    src = tmp_path / "drv.cpp"
    src.write_text(DRIVER)
    exe = tmp_path / "drv"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(ROOT, "biped_pympc_amd", "csrc"),
                    "-o", str(exe), str(src), "-lpthread"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
