#include "host_loader.h"

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <stdexcept>
#include <string>

namespace ea {

static void chk(hipError_t e, const char* w) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + w + ": " + hipGetErrorString(e));
}

HostLoader::HostLoader(long long chunk_bytes, int nbuf, int threads) : chunk_(chunk_bytes) {
  if (chunk_bytes <= 0 || nbuf < 1) throw std::invalid_argument("HostLoader: bad sizes");
  if (threads <= 0) {
    const char* e = getenv("ELEPHAS_AMD_LOADER_THREADS");
    threads = e ? atoi(e) : (int)std::min(8u, std::max(1u, std::thread::hardware_concurrency()));
  }
  threads_ = std::max(1, threads);
  for (int i = 0; i < nbuf; ++i) {
    void* p = nullptr;
    chk(hipHostMalloc(&p, (size_t)chunk_bytes, hipHostMallocDefault), "hipHostMalloc");
    bufs_.push_back(reinterpret_cast<char*>(p));
    hipEvent_t e;
    chk(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    evs_.push_back(e);
    busy_.push_back(false);
  }
}

HostLoader::~HostLoader() {
  for (size_t i = 0; i < bufs_.size(); ++i) {
    if (busy_[i]) (void)hipEventSynchronize(evs_[i]);
    (void)hipEventDestroy(evs_[i]);
    (void)hipHostFree(bufs_[i]);
  }
}

char* HostLoader::acquire(hipStream_t) {
  const int i = next_;
  if (busy_[i]) chk(hipEventSynchronize(evs_[i]), "loader wait");  // DMA of this buffer finished
  busy_[i] = false;
  return bufs_[i];
}

void HostLoader::release(hipStream_t s) {
  chk(hipEventRecord(evs_[next_], s), "loader record");
  busy_[next_] = true;
  next_ = (next_ + 1) % (int)bufs_.size();
}

void HostLoader::upload(const void* host, void* dev, long long nbytes, hipStream_t s) {
  const char* h = reinterpret_cast<const char*>(host);
  char* d = reinterpret_cast<char*>(dev);
  for (long long off = 0; off < nbytes; off += chunk_) {
    const long long n = std::min(chunk_, nbytes - off);
    char* buf = acquire(s);
    const long long pg = 4096, full = n / pg * pg;  // split contiguous bytes into 4 KB rows
    pack(buf, h + off, pg, pg, full / pg);
    if (n > full) std::memcpy(buf + full, h + off + full, (size_t)(n - full));
    chk(hipMemcpyAsync(d + off, buf, (size_t)n, hipMemcpyHostToDevice, s), "loader H2D");
    release(s);
    bytes_ += n;
  }
}

// branch-free so the packing loop vectorises
static inline uint16_t bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  const uint32_t rne = (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
  const uint32_t qnan = (u >> 16) | 0x40u;
  return (uint16_t)((u & 0x7FFFFFFFu) > 0x7F800000u ? qnan : rne);
}

void HostLoader::pack(char* buf, const char* host, long long host_ld, long long row_bytes, long long nr,
                      bool cvt) const {
  auto part = [&](long long r0, long long r1) {
    if (cvt) {
      const long long nc = row_bytes / 2;
      for (long long r = r0; r < r1; ++r) {
        const float* src = reinterpret_cast<const float*>(host + r * host_ld);
        uint16_t* dst = reinterpret_cast<uint16_t*>(buf + r * row_bytes);
        for (long long c = 0; c < nc; ++c) dst[c] = bf16_rne(src[c]);
      }
    } else if (host_ld == row_bytes) {
      std::memcpy(buf + r0 * row_bytes, host + r0 * host_ld, (size_t)((r1 - r0) * row_bytes));
    } else {
      for (long long r = r0; r < r1; ++r) std::memcpy(buf + r * row_bytes, host + r * host_ld, (size_t)row_bytes);
    }
  };
  // one thread per 256 KB of the chunk (a 1 MB chunk uses up to 4): below that a
  // thread costs more to start than its share of the copy
  const int nt = (int)std::min<long long>(threads_, std::max<long long>(1, (nr * row_bytes) >> 18));
  last_nt_ = nt;
  if (nt <= 1) {
    part(0, nr);
    return;
  }
  std::vector<std::thread> ts;
  ts.reserve(nt - 1);
  for (int i = 1; i < nt; ++i) ts.emplace_back(part, nr * i / nt, nr * (i + 1) / nt);
  part(0, nr / nt);
  for (auto& t : ts) t.join();
}

void HostLoader::upload_rows(const char* host, long long host_ld, char* dev, long long dev_ld, long long nrows,
                             long long row_bytes, hipStream_t s) {
  rows_(host, host_ld, dev, dev_ld, nrows, row_bytes, false, s);
}

void HostLoader::upload_rows_bf16(const float* host, long long host_ld, char* dev, long long dev_ld, long long nrows,
                                  long long ncols, hipStream_t s) {
  rows_(reinterpret_cast<const char*>(host), host_ld, dev, dev_ld, nrows, 2 * ncols, true, s);
}

void HostLoader::rows_(const char* host, long long host_ld, char* dev, long long dev_ld, long long nrows,
                       long long row_bytes, bool cvt, hipStream_t s) {
  if (row_bytes > chunk_) throw std::invalid_argument("row larger than loader chunk");
  const long long rows_per_chunk = std::max<long long>(1, chunk_ / row_bytes);
  for (long long r0 = 0; r0 < nrows; r0 += rows_per_chunk) {
    const long long nr = std::min(rows_per_chunk, nrows - r0);
    char* buf = acquire(s);
    pack(buf, host + r0 * host_ld, host_ld, row_bytes, nr, cvt);
    chk(hipMemcpy2DAsync(dev + r0 * dev_ld, (size_t)dev_ld, buf, (size_t)row_bytes, (size_t)row_bytes, (size_t)nr,
                         hipMemcpyHostToDevice, s),
        "loader H2D 2D");
    release(s);
    bytes_ += nr * row_bytes;
  }
}

}  // namespace ea
