// Host allocator for the chip-table builder's multi-GB arrays: allocations of 2 MiB and
// more are 2 MiB aligned and advised for transparent huge pages, so first touch faults
// once per 2 MiB instead of once per 4 KiB (on C3's 5.3 GB table the 4 KiB faults cost
// more than the work that fills the arrays: profiles/r5/blob_upload_c3.txt).
#pragma once
#include <stdlib.h>
#include <sys/mman.h>

#include <cstddef>
#include <new>

#ifndef MGPU_HUGE_MIN
#define MGPU_HUGE_MIN (std::size_t(2) << 20)
#endif
namespace mgpu {

template <class T>
struct HugeAlloc {
  using value_type = T;
  HugeAlloc() = default;
  template <class U>
  HugeAlloc(const HugeAlloc<U>&) {}
  T* allocate(std::size_t n) {
    constexpr std::size_t kHuge = std::size_t(2) << 20;
    const std::size_t bytes = n * sizeof(T);
    void* p;
    if (bytes >= MGPU_HUGE_MIN) {
      const std::size_t al = (bytes + kHuge - 1) & ~(kHuge - 1);
      p = aligned_alloc(kHuge, al);
      if (p) madvise(p, al, MADV_HUGEPAGE);  // (advice only: ignored where THP is off)
    } else {
      p = malloc(bytes ? bytes : 1);
    }
    if (!p) throw std::bad_alloc();
    return static_cast<T*>(p);
  }
  void deallocate(T* p, std::size_t) noexcept { free(p); }
  template <class U>
  bool operator==(const HugeAlloc<U>&) const noexcept { return true; }
  template <class U>
  bool operator!=(const HugeAlloc<U>&) const noexcept { return false; }
};

}  // namespace mgpu
