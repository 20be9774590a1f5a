#include "host_loader.h"

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "executor.h"

namespace ea {

static void chk(hipError_t e, const char* w) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + w + ": " + hipGetErrorString(e));
}

HostLoader::HostLoader(long long chunk_bytes, int nbuf, int threads) : chunk_(chunk_bytes) {
  if (chunk_bytes <= 0 || nbuf < 1) throw std::invalid_argument("HostLoader: bad sizes");
  if (threads <= 0) {
    const char* e = getenv("ELEPHAS_AMD_LOADER_THREADS");
    // 16: a GPU's CPU share on an MI355X node (8 GPUs per host); the fp32 -> bf16 row
    // packing of inference inputs is bound by it (Wide predict)
    threads = e ? atoi(e) : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
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
  for (int i = 1; i < threads_; ++i) pool_.emplace_back(&HostLoader::worker, this, i);
}

HostLoader::~HostLoader() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : pool_) t.join();
  for (size_t i = 0; i < bufs_.size(); ++i) {
    if (busy_[i]) (void)hipEventSynchronize(evs_[i]);
    (void)hipEventDestroy(evs_[i]);
    (void)hipHostFree(bufs_[i]);
  }
}

// Pool thread `id` runs part `id` of every job that has more than `id` parts.
void HostLoader::worker(int id) {
  long long seen = 0;
  for (;;) {
    const std::function<void(int)>* job;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      if (id >= job_parts_) continue;
      job = job_;
    }
    (*job)(id);
    {
      std::lock_guard<std::mutex> g(mu_);
      if (--pending_ == 0) done_cv_.notify_one();
    }
  }
}

void HostLoader::run_parts(const std::function<void(int)>& f, int n) {
  if (n <= 1) {
    f(0);
    return;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    job_ = &f;
    job_parts_ = n;
    pending_ = n - 1;
    ++gen_;
  }
  cv_.notify_all();
  f(0);
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return pending_ == 0; });
  job_ = nullptr;
}

char* HostLoader::acquire() {
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
  const long long pg = 4096, full = nbytes / pg * pg;  // contiguous bytes as 4 KB rows + a tail
  if (full) rows_(reinterpret_cast<const char*>(host), pg, reinterpret_cast<char*>(dev), pg, full / pg, pg, false, s);
  if (nbytes > full) {
    char* buf = acquire();
    std::memcpy(buf, reinterpret_cast<const char*>(host) + full, (size_t)(nbytes - full));
    chk(hipMemcpyAsync(reinterpret_cast<char*>(dev) + full, buf, (size_t)(nbytes - full), hipMemcpyHostToDevice, s),
        "loader H2D");
    release(s);
    bytes_ += nbytes - full;
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

// one row fp32 -> bf16; compiled for AVX-512 / AVX2 / baseline and picked at run time
// (the default x86-64 build vectorises the branch-free loop only 4 wide)
#ifndef __HIP_DEVICE_COMPILE__   // host code: the gfx950 pass of this file has no x86 targets
__attribute__((target_clones("avx512f", "avx2", "default")))
#endif
static void cvt_row_bf16(const float* __restrict__ src, uint16_t* __restrict__ dst, long long nc) {
  for (long long c = 0; c < nc; ++c) dst[c] = bf16_rne(src[c]);
}

void HostLoader::pack(char* buf, const char* host, long long host_ld, long long row_bytes, long long nr, bool cvt) {
  auto part = [&](long long r0, long long r1) {
    if (cvt) {
      const long long nc = row_bytes / 2;
      for (long long r = r0; r < r1; ++r)
        cvt_row_bf16(reinterpret_cast<const float*>(host + r * host_ld), reinterpret_cast<uint16_t*>(buf + r * row_bytes),
                     nc);
    } else if (host_ld == row_bytes) {
      std::memcpy(buf + r0 * row_bytes, host + r0 * host_ld, (size_t)((r1 - r0) * row_bytes));
    } else {
      for (long long r = r0; r < r1; ++r) std::memcpy(buf + r * row_bytes, host + r * host_ld, (size_t)row_bytes);
    }
  };
  // one part per 256 KB of the chunk (a 1 MB chunk uses up to 4): below that the
  // hand-off costs more than the part's share of the copy
  const int nt = (int)std::min<long long>(threads_, std::max<long long>(1, (nr * row_bytes) >> 18));
  last_nt_ = nt;
  const std::function<void(int)> f = [&](int i) { part(nr * i / nt, nr * (i + 1) / nt); };
  run_parts(f, nt);
}

void HostLoader::copy_out(void* dst, const void* src, long long nbytes) {
  const int nt = (int)std::min<long long>(threads_, std::max<long long>(1, nbytes >> 18));
  const std::function<void(int)> f = [&](int i) {
    const long long a = nbytes * i / nt / 64 * 64, b = i + 1 == nt ? nbytes : nbytes * (i + 1) / nt / 64 * 64;
    std::memcpy(reinterpret_cast<char*>(dst) + a, reinterpret_cast<const char*>(src) + a, (size_t)(b - a));
  };
  run_parts(f, nt);
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
    char* buf = acquire();
    pack(buf, host + r0 * host_ld, host_ld, row_bytes, nr, cvt);
    if (dev_ld == row_bytes)  // dense destination rows: one linear DMA
      chk(hipMemcpyAsync(dev + r0 * dev_ld, buf, (size_t)(nr * row_bytes), hipMemcpyHostToDevice, s), "loader H2D");
    else
      chk(hipMemcpy2DAsync(dev + r0 * dev_ld, (size_t)dev_ld, buf, (size_t)row_bytes, (size_t)row_bytes, (size_t)nr,
                           hipMemcpyHostToDevice, s),
          "loader H2D 2D");
    release(s);
    bytes_ += nr * row_bytes;
  }
}

namespace {
// a host range pinned for the duration of one call (owned: this call registered it)
struct HostPin {
  void* p = nullptr;
  bool owned = false;
  HostPin(const void* ptr, size_t bytes) {
    if (!ptr || !bytes) return;
    const hipError_t e = hipHostRegister(const_cast<void*>(ptr), bytes, hipHostRegisterDefault);
    if (e == hipSuccess) {
      p = const_cast<void*>(ptr);
      owned = true;
    } else {
      (void)hipGetLastError();
      if (e == hipErrorHostMemoryAlreadyRegistered) p = const_cast<void*>(ptr);
    }
  }
  ~HostPin() {
    if (owned) (void)hipHostUnregister(p);
  }
  explicit operator bool() const { return p != nullptr; }
};
}  // namespace

extern "C" hipError_t ea_cvt_rows_bf16(const float* src, long long src_ld, void* dst, long long dst_ld, long long nr,
                                       long long k, hipStream_t s);

void infer_pipeline(Executor& exe, HostLoader& L, const InferPipeArgs& a, const EvalSource& src, hipStream_t s_up,
                    hipStream_t s_comp, hipStream_t s_down) {
  if (a.n <= 0) return;
  if (a.B <= 0 || a.stage_rows <= 0 || a.stage_rows % a.B) throw std::invalid_argument("infer_pipeline: bad stage");
  if (a.x_bf16 && !a.dStage) throw std::invalid_argument("infer_pipeline: bf16 rows need a device staging buffer");
  const long long nst = (a.n + a.stage_rows - 1) / a.stage_rows;
  // bf16 rows: by default the packing threads convert on the host (half the PCIe bytes);
  // ELEPHAS_AMD_INFER_DEVICE_CVT=1: pin the fp32 rows, DMA them (one linear copy when
  // dense) and convert on the device
  const char* dc = std::getenv("ELEPHAS_AMD_INFER_DEVICE_CVT");
  const bool dev_cvt = a.x_bf16 && dc && std::atoi(dc) != 0;
  const HostPin xpin((a.x_bf16 && !dev_cvt) ? nullptr : a.x, (size_t)(((a.n - 1) * a.x_ld + a.k) * 4));
  const HostPin ypin(a.y, a.y ? (size_t)(((a.n - 1) * a.y_ld + a.ky) * 4) : 0);
  const HostPin opin(a.out, a.out ? (size_t)(a.n * a.ldp * 4) : 0);
  std::vector<hipEvent_t> evs;  // [up, done] + one download event per stage (staged copy-out)
  auto mk = [&]() {
    hipEvent_t e;
    chk(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    evs.push_back(e);
    return e;
  };
  const bool out_direct = a.out && opin;
  long long copied = 0;  // stages whose predictions are in `out` (staged copy-out)
  auto copy_stage = [&](long long st) {
    const long long lo = st * a.stage_rows, nr = std::min(a.stage_rows, a.n - lo);
    L.copy_out(a.out + lo * a.ldp, a.hPred + lo * a.ldp, nr * a.ldp * 4);
  };
  try {
    hipEvent_t up = mk(), done = mk();
    std::vector<hipEvent_t> dn;
    for (long long st = 0; st < nst; ++st) {
      const long long lo = st * a.stage_rows, nr = std::min(a.stage_rows, a.n - lo);
      const float* xh = a.x + lo * a.x_ld;
      if (xpin && a.x_bf16) {
        if (a.x_ld == a.k)   // dense rows: one linear DMA (the 2D path is a slower copy)
          chk(hipMemcpyAsync(a.dStage, xh, (size_t)(nr * a.k * 4), hipMemcpyHostToDevice, s_up), "infer H2D");
        else
          chk(hipMemcpy2DAsync(a.dStage, (size_t)(a.k * 4), xh, (size_t)(a.x_ld * 4), (size_t)(a.k * 4), (size_t)nr,
                               hipMemcpyHostToDevice, s_up),
              "infer H2D");
        chk(ea_cvt_rows_bf16(a.dStage, a.k, a.dX + lo * a.dX_ld, a.dX_ld / 2, nr, a.k, s_up), "infer cvt");
      } else if (xpin) {
        chk(hipMemcpy2DAsync(a.dX + lo * a.dX_ld, (size_t)a.dX_ld, xh, (size_t)(a.x_ld * 4), (size_t)(a.k * 4),
                             (size_t)nr, hipMemcpyHostToDevice, s_up),
            "infer H2D");
      } else if (a.x_bf16) {
        L.upload_rows_bf16(xh, a.x_ld * 4, a.dX + lo * a.dX_ld, a.dX_ld, nr, a.k, s_up);
      } else {
        L.upload_rows(reinterpret_cast<const char*>(xh), a.x_ld * 4, a.dX + lo * a.dX_ld, a.dX_ld, nr, a.k * 4, s_up);
      }
      if (a.y) {
        const float* yh = a.y + lo * a.y_ld;
        if (ypin)
          chk(hipMemcpy2DAsync(a.dY + lo * a.dY_ld, (size_t)(a.dY_ld * 4), yh, (size_t)(a.y_ld * 4), (size_t)(a.ky * 4),
                               (size_t)nr, hipMemcpyHostToDevice, s_up),
              "infer H2D y");
        else
          L.upload_rows(reinterpret_cast<const char*>(yh), a.y_ld * 4, reinterpret_cast<char*>(a.dY + lo * a.dY_ld),
                        a.dY_ld * 4, nr, a.ky * 4, s_up);
      }
      chk(hipEventRecord(up, s_up), "hipEventRecord");
      chk(hipStreamWaitEvent(s_comp, up, 0), "hipStreamWaitEvent");
      for (long long c = lo / a.B; c * a.B < lo + nr; ++c) exe.eval_chunk(c, src, s_comp);
      if (a.hPred || out_direct) {
        chk(hipEventRecord(done, s_comp), "hipEventRecord");
        chk(hipStreamWaitEvent(s_down, done, 0), "hipStreamWaitEvent");
        float* dst = out_direct ? a.out : a.hPred;
        chk(hipMemcpyAsync(dst + lo * a.ldp, a.dPred + lo * a.ldp, (size_t)(nr * a.ldp * 4), hipMemcpyDeviceToHost,
                           s_down),
            "infer D2H");
        dn.push_back(mk());
        chk(hipEventRecord(dn.back(), s_down), "hipEventRecord");
        // staged results: finished stages -> `out` while later stages are in flight
        while (a.out && !out_direct && copied < st && hipEventQuery(dn[copied]) == hipSuccess) copy_stage(copied++);
      }
    }
    // the host arrays are unpinned on return: every transfer touching them must be done
    if (a.out && !dn.empty()) {
      if (out_direct) {
        chk(hipEventSynchronize(dn.back()), "hipEventSynchronize");
      } else {
        for (; copied < nst; ++copied) {
          chk(hipEventSynchronize(dn[copied]), "hipEventSynchronize");
          copy_stage(copied);
        }
      }
    }
    if (xpin.owned || ypin.owned) chk(hipEventSynchronize(up), "hipEventSynchronize");
  } catch (...) {
    (void)hipStreamSynchronize(s_up);
    (void)hipStreamSynchronize(s_down);
    for (auto e : evs) (void)hipEventDestroy(e);
    throw;
  }
  // destroying a recorded event is legal: its pending waits stay valid
  for (auto e : evs) (void)hipEventDestroy(e);
}

}  // namespace ea
