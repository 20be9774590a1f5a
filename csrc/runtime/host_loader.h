// Host -> device data loader with pinned, multi-buffered staging.
//
// Replaces Spark's parallelize/repartition data shipping (reference
// utils/rdd_utils.py:10-20, spark_model.py:182-183): a rank's partition
// (contiguous rows of the host dataset) is streamed into HBM through `nbuf`
// pinned chunks; a persistent pool of packing threads copies (or converts to
// bf16) chunk i+1 into pinned memory while the DMA engine moves chunk i (one
// thread's memcpy into pinned memory runs at ~5-10 GB/s, below the DMA rate).
// Sized for 288 GB HBM: whole shards stay resident on the device afterwards.
//
// infer_pipeline (below) runs inference over host rows as a three-stream
// pipeline on top of the loader: uploads on one stream, the eval executor's
// kernels on a second, prediction downloads on a third, ordered by events.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace ea {

class Executor;
struct EvalSource;

class HostLoader {
 public:
  // threads: CPU threads packing each chunk (0 = $ELEPHAS_AMD_LOADER_THREADS or min(8, cores))
  HostLoader(long long chunk_bytes, int nbuf = 3, int threads = 0);
  ~HostLoader();
  HostLoader(const HostLoader&) = delete;
  HostLoader& operator=(const HostLoader&) = delete;
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
  long long chunk_bytes() const { return chunk_; }
  // host memcpy split over the packing pool (pinned staging -> pageable results)
  void copy_out(void* dst, const void* src, long long nbytes);

 private:
  long long chunk_;
  int threads_ = 1;
  mutable int last_nt_ = 0;
  // cvt: host rows are fp32 and buf rows bf16 (row_bytes = 2 * columns)
  void pack(char* buf, const char* host, long long host_ld, long long row_bytes, long long nr, bool cvt = false);
  void rows_(const char* host, long long host_ld, char* dev, long long dev_ld, long long nrows, long long row_bytes,
             bool cvt, hipStream_t s);
  std::vector<char*> bufs_;
  std::vector<hipEvent_t> evs_;
  std::vector<bool> busy_;
  long long bytes_ = 0;
  int next_ = 0;
  char* acquire();
  void release(hipStream_t s);
  // persistent packing pool: run(f, n) calls f(0..n-1) with part 0 on the caller
  void run_parts(const std::function<void(int)>& f, int n);
  void worker(int id);
  std::vector<std::thread> pool_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* job_ = nullptr;
  int job_parts_ = 0;
  long long gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
};

struct InferPipeArgs {
  const float* x = nullptr; long long x_ld = 0, n = 0, k = 0;   // host feature rows (fp32)
  char* dX = nullptr; long long dX_ld = 0; int x_bf16 = 0;       // device rows (bytes stride)
  const float* y = nullptr; long long y_ld = 0, ky = 0;          // optional host targets (fp32)
  float* dY = nullptr; long long dY_ld = 0;                      // device targets (floats stride)
  float* dPred = nullptr; long long ldp = 0; float* hPred = nullptr;  // optional predictions (pinned)
  float* out = nullptr;                                          // optional: predictions copied here too
  float* dStage = nullptr;                                       // bf16 x: fp32 device staging, stage_rows x k
  long long stage_rows = 0;                                      // rows per stage (multiple of B)
  int B = 0;                                                     // the eval executor's chunk rows
};

// The host arrays x, y and out are pinned in place for the call (hipHostRegister,
// ~0.8 ms for 200 MB) so every transfer is a direct DMA from / to them (bf16 x: fp32
// rows DMA'd into dStage and converted on the device); where pinning is refused the
// loader's packing threads stage through pinned buffers instead.
// Stage s: upload its rows (+ targets) on s_up -> event -> the eval chunks of those
// rows on s_comp -> event -> download their predictions into pinned host memory on
// s_down. The host packs stage s+1 while the GPU computes stage s, and copies the
// pinned predictions of finished stages into `out` (pageable) with the packing pool
// in between. Returns after every stage's predictions are in `out` (when given).
void infer_pipeline(Executor& exe, HostLoader& L, const InferPipeArgs& a, const EvalSource& src,
                    hipStream_t s_up, hipStream_t s_comp, hipStream_t s_down);

}  // namespace ea
