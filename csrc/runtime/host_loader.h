// Host -> device data loader with pinned, double-buffered staging.
//
// Replaces Spark's parallelize/repartition data shipping (reference
// utils/rdd_utils.py:10-20, spark_model.py:182-183): a rank's partition
// (contiguous rows of the host dataset) is streamed into HBM through `nbuf`
// pinned chunks; the CPU packs chunk i+1 (several threads: one thread's memcpy
// into pinned memory runs at ~5 GB/s, below the DMA rate) while the DMA engine
// moves chunk i.
// Sized for 288 GB HBM: whole shards stay resident on the device afterwards.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

namespace ea {

class HostLoader {
 public:
  // threads: CPU threads packing each chunk (0 = $ELEPHAS_AMD_LOADER_THREADS or min(8, cores))
  HostLoader(long long chunk_bytes, int nbuf = 2, int threads = 0);
  ~HostLoader();
  // contiguous copy
  void upload(const void* host, void* dev, long long nbytes, hipStream_t s);
  // row-strided copy (e.g. pad rows to a 16-byte multiple on the device)
  void upload_rows(const char* host, long long host_ld, char* dev, long long dev_ld, long long nrows,
                   long long row_bytes, hipStream_t s);
  // fp32 rows -> bf16 rows (round to nearest even, NaN kept quiet), converted by the
  // packing threads: half the PCIe bytes of staging fp32 and converting on the device
  void upload_rows_bf16(const float* host, long long host_ld, char* dev, long long dev_ld, long long nrows,
                        long long ncols, hipStream_t s);
  long long bytes_uploaded() const { return bytes_; }
  int threads() const { return threads_; }
  // threads the most recent chunk was packed with (diagnostics / tests)
  int last_pack_threads() const { return last_nt_; }

 private:
  long long chunk_;
  int threads_ = 1;
  mutable int last_nt_ = 0;
  // rows [0, nr) of `host` (stride host_ld) -> dense rows in `buf`, split over threads_
  // cvt: host rows are fp32 and buf rows bf16 (row_bytes = 2 * columns)
  void pack(char* buf, const char* host, long long host_ld, long long row_bytes, long long nr, bool cvt = false) const;
  void rows_(const char* host, long long host_ld, char* dev, long long dev_ld, long long nrows, long long row_bytes,
             bool cvt, hipStream_t s);
  std::vector<char*> bufs_;
  std::vector<hipEvent_t> evs_;
  std::vector<bool> busy_;
  long long bytes_ = 0;
  int next_ = 0;
  char* acquire(hipStream_t s);
  void release(hipStream_t s);
};

}  // namespace ea
