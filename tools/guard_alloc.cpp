// Diagnostic allocator for torch (torch.cuda.memory.CUDAPluggableAllocator): every block gets
// a 1 MiB guard zone before and after it, and the guards (and, unless GUARD_POISON_BODY=0,
// the block itself) are filled with 0xFFFFFFFF per 32-bit word: NaN as f32, -1 as an int32
// index.  A kernel that READS past either end of a tensor, or reads memory nobody wrote, then
// sees NaN (an index: -1, whose row lies in the guard before the block) instead of whatever
// the neighbouring allocation held; a kernel that WRITES past either end leaves non-poison
// words in a guard, which guard_check() finds (tools/oob_hunt.py calls it after every op).
// No caching: hipMalloc / hipFree per block (slow; diagnostics only).
//
//   hipcc -O2 -shared -fPIC tools/guard_alloc.cpp -o tools/guard_alloc.so
#include <hip/hip_runtime.h>
#include <sys/types.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace {
constexpr size_t kGuard = 1 << 20;   // 1 MiB before and after (keeps 2 MiB alignment)
constexpr size_t kCheck = 16 << 10;  // guard bytes next to the block that guard_check reads
constexpr unsigned kPoison = 0xFFFFFFFFu;

bool poison_body() {
  static const bool on = [] {
    const char* e = getenv("GUARD_POISON_BODY");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

struct Live {
  size_t body;
  int device;
};
std::mutex mu;
std::unordered_map<char*, Live> live;  // body pointer -> size
std::string report;

#define CK(x) (void)(x)

// first non-poison word of n bytes at device address p, or -1
long first_bad(const char* p, size_t n, std::vector<unsigned>& buf) {
  buf.resize(n / 4);
  CK(hipMemcpy(buf.data(), p, n, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < buf.size(); ++i)
    if (buf[i] != kPoison) return (long)i;
  return -1;
}
}  // namespace

extern "C" {

void* guard_malloc(ssize_t size, int device, hipStream_t stream) {
  (void)stream;
  int prev = 0;
  CK(hipGetDevice(&prev));
  CK(hipSetDevice(device));
  const size_t body = ((size_t)size + 255) & ~(size_t)255;
  char* base = nullptr;
  if (hipMalloc(&base, body + 2 * kGuard) != hipSuccess) {
    CK(hipSetDevice(prev));
    return nullptr;
  }
  if (poison_body()) {
    CK(hipMemsetD32((hipDeviceptr_t)base, kPoison, (body + 2 * kGuard) / 4));
  } else {
    CK(hipMemsetD32((hipDeviceptr_t)base, kPoison, kGuard / 4));
    CK(hipMemsetD32((hipDeviceptr_t)(base + kGuard + body), kPoison, kGuard / 4));
  }
  CK(hipDeviceSynchronize());
  CK(hipSetDevice(prev));
  std::lock_guard<std::mutex> g(mu);
  live[base + kGuard] = Live{body, device};
  return base + kGuard;
}

void guard_free(void* ptr, ssize_t size, int device, hipStream_t stream) {
  (void)size;
  (void)stream;
  if (ptr == nullptr) return;
  int prev = 0;
  CK(hipGetDevice(&prev));
  CK(hipSetDevice(device));
  CK(hipDeviceSynchronize());
  {
    std::lock_guard<std::mutex> g(mu);
    live.erase((char*)ptr);
  }
  CK(hipFree((char*)ptr - kGuard));
  CK(hipSetDevice(prev));
}

// Check the kCheck guard bytes on both sides of every live block.  Returns the number of
// blocks with a clobbered guard; guard_report() then describes them.  Reported guards are
// re-poisoned, so the next call reports only new writes.
int guard_check(void) {
  CK(hipDeviceSynchronize());
  std::lock_guard<std::mutex> g(mu);
  std::vector<unsigned> buf;
  int bad = 0;
  report.clear();
  for (auto& kv : live) {
    char* p = kv.first;
    const size_t body = kv.second.body;
    const long lo = first_bad(p - kCheck, kCheck, buf);
    const long hi = first_bad(p + body, kCheck, buf);
    if (lo < 0 && hi < 0) continue;
    ++bad;
    char line[256];
    snprintf(line, sizeof line, "block %p (%zu bytes): %s%s\n", (void*)p, body,
             lo >= 0 ? "written BEFORE its start " : "",
             hi >= 0 ? "written PAST its end " : "");
    report += line;
    if (hi >= 0) {
      snprintf(line, sizeof line, "   first clobbered word after the end: +%ld bytes\n", hi * 4);
      report += line;
    }
    if (lo >= 0) {
      snprintf(line, sizeof line, "   first clobbered word before the start: -%ld bytes\n",
               (long)kCheck - lo * 4);
      report += line;
    }
    CK(hipMemsetD32((hipDeviceptr_t)(p - kCheck), kPoison, kCheck / 4));
    CK(hipMemsetD32((hipDeviceptr_t)(p + body), kPoison, kCheck / 4));
  }
  CK(hipDeviceSynchronize());
  return bad;
}

const char* guard_report(void) { return report.c_str(); }

int guard_live(void) {
  std::lock_guard<std::mutex> g(mu);
  return (int)live.size();
}

}  // extern "C"
