// ricepp_facade.cpp -- C++ host facade (include/ricepp_amd.hpp) over the C ABI.
//
// The DwarFS plugin semantics follow src/compression/ricepp.cpp (file:line
// cited at each method).  Encode / decode calls go through a per-(device,
// config, direction) pipelined batch queue: concurrent calls are coalesced
// into one rpp_encode_batch_ws / rpp_decode_batch_ws launch on a pooled device
// context (stream + event + device buffers + mapped pinned staging), so the
// worker_group threads of the DwarFS writer (src/writer/filesystem_writer.cpp:
// 255-287) and block cache (src/reader/internal/block_cache.cpp:628-706) feed
// the GPU in batches without any per-call stream creation or allocation.
#include "ricepp_amd.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <charconv>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <utility>
#include <vector>

namespace ricepp_amd {

namespace {

void hip_check(hipError_t e, char const* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("ricepp_amd: ") + what + ": " + hipGetErrorString(e));
}

rpp_config to_rpp(codec_config const& c) {
  rpp_config r{};
  r.block_size = c.block_size > 0xFFFFFFFFu ? 0xFFFFFFFFu : static_cast<uint32_t>(c.block_size);
  r.component_stream_count =
      c.component_stream_count > 0xFFFFFFFFu ? 0xFFFFFFFFu : static_cast<uint32_t>(c.component_stream_count);
  r.big_endian = c.byteorder == std::endian::big ? 1u : 0u;
  r.unused_lsb_count = c.unused_lsb_count;
  return r;
}

[[noreturn]] void throw_status(int st) {
  switch (st) {
    case RPP_UNSUPPORTED_CONFIG: throw std::runtime_error("Unsupported configuration");
    case RPP_TRUNCATED_INPUT: throw std::out_of_range("bitstream_reader::read_packet");
    case RPP_INVALID_ARGUMENT: throw std::invalid_argument("ricepp_amd: invalid argument");
    case RPP_OUTPUT_TOO_SMALL: throw std::length_error("ricepp_amd: output buffer too small");
    case RPP_INTERNAL_ERROR: throw std::runtime_error("ricepp_amd: internal error (device consistency bound)");
    default: throw std::runtime_error("ricepp_amd: HIP error");
  }
}

size_t align16(size_t v) { return (v + 15) & ~size_t{15}; }

std::atomic<uint64_t> g_enc_launches{0}, g_enc_blocks{0}, g_dec_launches{0}, g_dec_blocks{0}, g_ctx_created{0},
    g_buffer_grows{0}, g_buffer_grow_ns{0};
std::atomic<uint32_t> g_ctx_faults{0};     // inject_context_failures
std::atomic<uint32_t> g_launch_faults{0};  // inject_launch_failures
// a test hook: throws once per injected launch failure
void maybe_fail_launch() {
  for (uint32_t n = g_launch_faults.load(); n;)
    if (g_launch_faults.compare_exchange_weak(n, n - 1)) throw std::runtime_error("ricepp_amd: injected launch failure");
}
std::atomic<uint64_t> g_stage_ns{0}, g_device_ns{0}, g_finish_ns{0}, g_device_event_ns{0};
// set once shutdown_facade() has begun: the context pool makes no more HIP
// calls (contexts returned afterwards are leaked, new ones refused)
std::atomic<bool> g_shutdown{false};
inline uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
// batch trace (set_facade_trace): records appended when a batch is released
std::atomic<bool> g_trace_on{false};
std::mutex g_trace_mu;
std::vector<facade_batch_record> g_trace;

int current_device() {
  int d = 0;
  hip_check(hipGetDevice(&d), "hipGetDevice");
  return d;
}

// Makes `dev` current for the calling thread for the guard's lifetime.
class device_guard {
 public:
  explicit device_guard(int dev) : dev_{dev} {
    hip_check(hipGetDevice(&prev_), "hipGetDevice");
    if (prev_ != dev_) hip_check(hipSetDevice(dev_), "hipSetDevice");
  }
  ~device_guard() {
    if (prev_ != dev_) (void)hipSetDevice(prev_);
  }
  device_guard(device_guard const&) = delete;
  device_guard& operator=(device_guard const&) = delete;

 private:
  int dev_;
  int prev_ = 0;
};

// A private stream plus device and pinned host buffers, bound to one device.
// Device buffers come from hipMalloc and grow geometrically while the context
// is idle (not from the stream-ordered allocator: with hipMallocAsync /
// hipFreeAsync, on the default pool or a pool per context, buffers of
// concurrent streams were overwritten -- tools/h2d_stress.hip reproduces it
// outside the library, 4 threads x 128 MiB; hipMalloc passes).  Pinned buffers are mapped into the device's address space (the
// encoder packs its output straight into them) and grow geometrically; a
// context going back to the pool drops pinned buffers above kPinnedKeep and
// device buffers above kDeviceKeep, so a burst of huge batches does not keep
// GiBs of host memory pinned or of device memory reserved.
constexpr size_t kPinnedKeep = size_t{320} << 20;  // (a batch of 8 x 16 MiB blocks: 128 + 64 MiB)
constexpr size_t kDeviceKeep = size_t{1} << 30;  // (hipFree synchronises: trims stay rare)

class device_ctx {
 public:
  // kind: the pool a context returns to (encode batches, decode batches,
  // PCM calls), so that a context keeps buffers sized for one use
  device_ctx(int dev, int kind) : dev_{dev}, kind_{kind} {
    for (uint32_t n = g_ctx_faults.load(); n;)
      if (g_ctx_faults.compare_exchange_weak(n, n - 1)) throw std::runtime_error("hipStreamCreate: injected failure");
    device_guard g{dev_};
    hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    // the batch's start and end on the device's clock; a host thread waiting
    // for the end blocks (hipEventBlockingSync) instead of spinning on a core
    // the callers need
    if (hipEventCreateWithFlags(&start_, hipEventDefault) != hipSuccess) {
      (void)hipStreamDestroy(stream_);
      throw std::runtime_error("ricepp_amd: hipEventCreateWithFlags failed");
    }
    if (hipEventCreateWithFlags(&event_, hipEventBlockingSync) != hipSuccess) {
      (void)hipEventDestroy(start_);
      (void)hipStreamDestroy(stream_);
      throw std::runtime_error("ricepp_amd: hipEventCreateWithFlags failed");
    }
    g_ctx_created.fetch_add(1, std::memory_order_relaxed);
  }
  device_ctx(device_ctx const&) = delete;
  device_ctx& operator=(device_ctx const&) = delete;

  int device() const { return dev_; }
  int kind() const { return kind_; }
  hipStream_t stream() const { return stream_; }
  hipEvent_t event() const { return event_; }
  hipEvent_t start_event() const { return start_; }
  uint8_t* dev(size_t bytes) { return grow_dev(dbuf_, dcap_, bytes); }
  uint8_t* workspace(size_t bytes) { return grow_dev(wbuf_, wcap_, bytes); }
  uint8_t* pin_in(size_t bytes) { return grow_pinned(hin_, hin_cap_, bytes); }
  uint8_t* pin_out(size_t bytes) { return grow_pinned(hout_, hout_cap_, bytes); }
  size_t pinned_capacity() const { return hin_cap_ + hout_cap_; }
  bool pinned_fits(size_t in, size_t out) const { return hin_ && hout_ && in <= hin_cap_ && out <= hout_cap_; }
  // the device-side address of a pinned buffer
  uint8_t* device_view(uint8_t* pinned) {
    void* d = nullptr;
    hip_check(hipHostGetDevicePointer(&d, pinned, 0), "hipHostGetDevicePointer");
    return static_cast<uint8_t*>(d);
  }
  void sync() { hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize"); }
  // Waits for everything enqueued on the stream (a failed launch may have
  // left copies or kernels on it that still use the buffers); false if the
  // stream is in error, and the context must not be used again.
  bool drain() { return hipStreamSynchronize(stream_) == hipSuccess; }
  // frees everything (a context whose stream failed; errors ignored)
  void destroy() {
    for (uint8_t* q : {hin_, hout_})
      if (q) (void)hipHostFree(q);
    for (uint8_t* q : {dbuf_, wbuf_})
      if (q) (void)hipFree(q);
    (void)hipEventDestroy(event_);
    (void)hipEventDestroy(start_);
    (void)hipStreamDestroy(stream_);
    hin_ = hout_ = dbuf_ = wbuf_ = nullptr;
    hin_cap_ = hout_cap_ = dcap_ = wcap_ = 0;
  }
  // on release, after drain()
  void trim() {
    for (auto* q : {&hin_, &hout_}) {
      size_t& cap = q == &hin_ ? hin_cap_ : hout_cap_;
      if (cap > kPinnedKeep) {
        (void)hipHostFree(*q);
        *q = nullptr;
        cap = 0;
      }
    }
    for (auto* q : {&dbuf_, &wbuf_}) {
      size_t& cap = q == &dbuf_ ? dcap_ : wcap_;
      if (cap > kDeviceKeep) {
        (void)hipFree(*q);
        *q = nullptr;
        cap = 0;
      }
    }
  }

 private:
  uint8_t* grow_dev(uint8_t*& p, size_t& cap, size_t bytes) {
    if (bytes <= cap && p) return p;
    size_t n = cap ? cap : size_t{1} << 20;
    while (n < bytes) n *= 2;
    const uint64_t t0 = now_ns();
    if (p) (void)hipFree(p);  // (the context is idle: its last batch has completed)
    p = nullptr;
    cap = 0;
    void* q = nullptr;
    hip_check(hipMalloc(&q, n), "hipMalloc");
    g_buffer_grows.fetch_add(1, std::memory_order_relaxed);
    g_buffer_grow_ns.fetch_add(now_ns() - t0, std::memory_order_relaxed);
    p = static_cast<uint8_t*>(q);
    cap = n;
    return p;
  }
  // (pinned buffers only grow between batches: the stream is idle then)
  static uint8_t* grow_pinned(uint8_t*& p, size_t& cap, size_t bytes) {
    if (bytes <= cap && p) return p;
    size_t n = cap ? cap : size_t{1} << 20;
    while (n < bytes) n *= 2;
    const uint64_t t0 = now_ns();
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    void* q = nullptr;
    hip_check(hipHostMalloc(&q, n, hipHostMallocMapped), "hipHostMalloc");
    g_buffer_grows.fetch_add(1, std::memory_order_relaxed);
    g_buffer_grow_ns.fetch_add(now_ns() - t0, std::memory_order_relaxed);
    p = static_cast<uint8_t*>(q);
    cap = n;
    return p;
  }

  int dev_;
  int kind_;
  hipStream_t stream_ = nullptr;
  hipEvent_t event_ = nullptr;
  hipEvent_t start_ = nullptr;
  uint8_t* dbuf_ = nullptr;
  size_t dcap_ = 0;
  uint8_t* wbuf_ = nullptr;
  size_t wcap_ = 0;
  uint8_t* hin_ = nullptr;
  size_t hin_cap_ = 0;
  uint8_t* hout_ = nullptr;
  size_t hout_cap_ = 0;
};

// Per-device free lists of contexts (intentionally leaked at exit: no HIP
// calls from static destructors).
class ctx_pool {
 public:
  static ctx_pool& get() {
    static ctx_pool* p = new ctx_pool;
    return *p;
  }
  // kind: 0 encode batches, 1 decode batches, 2 other (PCM): encode and
  // decode size their device and pinned buffers differently, and a context
  // handed from one to the other regrew them (hipFree / hipHostFree
  // synchronise the device) -- one pool per kind keeps them grown
  // A batch asks for the pinned capacity it will use: the pooled context that
  // already holds enough and the least of it, else the one holding the most
  // (growing a buffer frees the old one first, which synchronises the
  // device: a 16 MiB-block batch regrowing 256 MiB of pinned memory stalled
  // both streams for ~70 ms, profiles/r06_facade_16m.jsonl).
  device_ctx* acquire(int dev, int kind, size_t pin_in = 0, size_t pin_out = 0) {
    if (g_shutdown.load(std::memory_order_acquire)) throw std::runtime_error("ricepp_amd: facade shut down");
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto& v = free_[{dev, kind}];
      if (!v.empty()) {
        size_t best = v.size() - 1;  // (the most recent: LIFO when nothing is asked)
        if (pin_in || pin_out) {
          for (size_t i = 0; i < v.size(); ++i) {
            const bool fi = v[i]->pinned_fits(pin_in, pin_out), fb = v[best]->pinned_fits(pin_in, pin_out);
            const size_t ci = v[i]->pinned_capacity(), cb = v[best]->pinned_capacity();
            if (fi != fb ? fi : (fi ? ci < cb : ci > cb)) best = i;
          }
        }
        device_ctx* c = v[best];
        v.erase(v.begin() + best);
        return c;
      }
    }
    return new device_ctx(dev, kind);
  }
  // Drains the context's stream (idle in the normal case: a batch ends with
  // its event; after a failed launch it may still hold work) and pools it,
  // or destroys it when its stream is in error.  Never called with a queue
  // lock held: the drain and the trim may synchronise.
  void release(device_ctx* c) {
    if (g_shutdown.load(std::memory_order_acquire)) return;  // (no HIP calls once shutting down: leaked)
    try {
      device_guard g{c->device()};
      if (!c->drain()) {
        c->destroy();
        delete c;
        return;
      }
      c->trim();
    } catch (...) {  // (hipSetDevice failed: the context cannot be trusted; freed, errors ignored)
      c->destroy();
      delete c;
      return;
    }
    std::lock_guard<std::mutex> lk(mu_);
    free_[{c->device(), c->kind()}].push_back(c);
  }

 private:
  std::mutex mu_;
  std::map<std::pair<int, int>, std::vector<device_ctx*>> free_;
};

class ctx_lease {
 public:
  explicit ctx_lease(int dev) : c_{ctx_pool::get().acquire(dev, 2)} {}
  ~ctx_lease() { ctx_pool::get().release(c_); }
  ctx_lease(ctx_lease const&) = delete;
  ctx_lease& operator=(ctx_lease const&) = delete;
  device_ctx& operator*() const { return *c_; }
  device_ctx* operator->() const { return c_; }

 private:
  device_ctx* c_;
};

// ---- pipelined batch queue ----
//
// DwarFS calls the codec synchronously from a pool of worker threads, one
// block per call (filesystem_writer.cpp:255-287, block_cache.cpp:628-706).
// Concurrent calls of one (device, configuration, direction) are gathered
// into batches, each batch one launch on a pooled context:
//   * a caller reserves its slot in the open batch's pinned staging and
//     copies its input in -- in parallel with the other callers, no waiting;
//   * the open batch is closed as soon as fewer than g_max_active batches are
//     on the device (an idle queue launches a lone call at once, a busy one
//     gathers everything that arrives meanwhile), or when it is full;
//   * the queue's driver thread launches a closed batch once every caller has
//     copied in (copies and kernels enqueued between two events);
//   * the queue's waiter thread blocks on the end event of the oldest batch
//     in flight (a blocking-sync event: no core spins), then takes every
//     other batch in flight that has finished too, and publishes each batch's
//     results with one wake-up of all its callers;
//   * every caller copies its own result out; the last one returns the
//     context to the pool.
// So a call costs one reservation, two copies and one futex wait, and the
// device keeps up to g_max_active batches in flight.  Callers make HIP calls
// only to bring up a batch (a pooled context, pinned staging) and to return
// its context to the pool, never with the queue's lock held; they never wait
// on the device.
struct batch;

struct request {
  // encode: in = samples, out = caller's output; decode: in = stream bytes,
  // out = sample bytes
  uint8_t const* in;
  size_t in_bytes;
  uint8_t* out;
  size_t out_cap;  // encode: output span size; decode: exact sample bytes
  uint64_t n_samples;
  // set by the queue (the results before the batch's `done` is raised)
  uint8_t* pin_in = nullptr;
  uint8_t const* pin_out = nullptr;
  size_t in_off = 0, out_off = 0;
  size_t result_bytes = 0;
  int status = RPP_OK;
  std::string error;  // HIP failure text
};

struct batch {
  device_ctx* ctx = nullptr;
  std::vector<request*> reqs;
  uint8_t* pin_in = nullptr;   // [inputs][parameter arrays]
  uint8_t* pin_out = nullptr;  // [outputs][sizes / statuses]
  size_t in_cap = 0, out_cap = 0;
  size_t in_fill = 0, out_fill = 0;  // reserved bytes (16-aligned slots)
  uint64_t total_samples = 0, max_samples = 0;
  size_t staged = 0;  // (mutex)
  bool closed = false;
  bool packed = true;  // encode: outputs packed back to back (else at their slots)
  std::atomic<uint32_t> done{0};      // results published (callers wait on it)
  std::atomic<size_t> finished{0};    // callers that have copied out
  size_t join = 1;  // requests of the opening one's size it was sized for
  uint64_t t_open = 0, t_close = 0, t_ready = 0, t_launch = 0, t_done = 0;
  int inflight_at_close = 0;
};

constexpr size_t kMaxBatchBlocks = 8192;
// pinned staging per batch (a larger single request gets a batch of its own size)
constexpr size_t kBatchIn = size_t{8} << 20;
constexpr size_t kBatchOut = size_t{16} << 20;
// A batch opened by a request larger than kBatchOut / 4 (DwarFS blocks of
// 4 MiB and up: mkdwarfs -S 22..30) has room for kLargeJoin requests of its
// size, so that concurrent long blocks share one segmented launch and its
// copies instead of one launch each (block_cache.cpp:628-706 issues them
// from a worker pool).
constexpr size_t kLargeJoin = 8;
// ... as long as the batch's staging stays within this (a 1 GiB block,
// mkdwarfs -S 29, gets a batch of its own: pinned staging of its size only)
constexpr size_t kLargeJoinBudget = size_t{256} << 20;
// encode batches whose worst-case output exceeds this go out by a DMA copy of
// the slots instead of being packed into mapped host memory by a kernel
// (set_facade_pack_limit changes it for benchmarks; default: always pack)
std::atomic<size_t> g_pack_max{~size_t{0}};
// batches of one queue on the device at once (set_facade_pipeline_depth
// changes it for benchmarks)
std::atomic<int> g_max_active{2};
// A batch of large requests (one opened with room for several, kLargeJoin)
// that a caller finishes staging while another batch is on the device closes
// only once it holds this many requests (else the completion of the batch on
// the device closes it): DwarFS-style worker pools finish a batch together
// and re-enter one by one, and closing at the first one's staging split them
// into uneven batches -- 8, 1, 7, 1, 8 ... of 16 MiB blocks
// (profiles/r06_facade_16m_*.jsonl).  set_facade_large_min_fill changes it.
std::atomic<int> g_large_min_fill{4};
// batches alive per queue beyond those on the device (open + being copied
// out); a caller that finds none with room waits for one to be released
constexpr int kSpareBatches = 2;

class batch_queue {
 public:
  batch_queue(int dev, rpp_config cfg, bool encode) : dev_{dev}, cfg_{cfg}, encode_{encode} {}

  void run(request& r) {
    std::unique_lock<std::mutex> lk(mu_);
    if (stopping_) throw std::runtime_error("ricepp_amd: facade shut down");
    if (!driver_.joinable()) {
      driver_ = std::thread([this] { drive(); });
      waiter_ = std::thread([this] { wait_loop(); });
    }
    ++active_;
    batch* b = nullptr;
    try {
      b = reserve(lk, r);
    } catch (...) {  // (nothing holds r yet; contexts parked by discard() are pooled all the same)
      std::vector<device_ctx*> parked;
      parked.swap(discarded_);
      leave(lk);
      lk.unlock();
      for (device_ctx* c : parked) ctx_pool::get().release(c);
      throw;
    }
    std::vector<device_ctx*> unused;
    unused.swap(discarded_);
    lk.unlock();
    for (device_ctx* c : unused) ctx_pool::get().release(c);
    if (r.in_bytes) std::memcpy(r.pin_in, r.in, r.in_bytes);
    lk.lock();
    ++b->staged;
    if (!b->closed && (stopping_ || (inflight_ < g_max_active.load(std::memory_order_relaxed) &&
                                     (inflight_ == 0 || b->join == 1 ||
                                      b->reqs.size() >= std::min<size_t>(b->join, (size_t)g_large_min_fill.load())))))
      close(b);
    else if (b->closed && b->staged == b->reqs.size()) make_ready(b);
    lk.unlock();
    while (!b->done.load(std::memory_order_acquire)) b->done.wait(0, std::memory_order_acquire);
    if (r.status == RPP_OK && r.result_bytes) std::memcpy(r.out, r.pin_out, r.result_bytes);
    device_ctx* c = nullptr;
    const bool last = b->finished.fetch_add(1, std::memory_order_acq_rel) + 1 == b->reqs.size();
    lk.lock();
    if (last) c = release(b);
    lk.unlock();
    if (c) ctx_pool::get().release(c);
    lk.lock();
    leave(lk);
  }

  // Stops the queue (shutdown_facade): batches in flight complete, batches
  // not launched fail, later calls throw; joins the queue's threads and
  // waits (bounded) for the callers inside run() to leave it.
  void shutdown() {
    std::unique_lock<std::mutex> lk(mu_);
    if (stopping_) return;
    stopping_ = true;
    // (an open batch whose callers have all copied in goes out now, and
    // fails; one still being copied into is closed by its last caller)
    if (open_ && !open_->reqs.empty() && open_->staged == open_->reqs.size()) close(open_);
    drv_cv_.notify_all();
    wait_cv_.notify_all();
    lk.unlock();
    if (driver_.joinable()) driver_.join();
    if (waiter_.joinable()) waiter_.join();
    lk.lock();
    quiet_cv_.wait_for(lk, std::chrono::seconds(5), [&] { return active_ == 0; });
  }

 private:
  static size_t arrays_in(size_t nb) { return 4 * nb * 8 + 64; }
  static size_t arrays_out(size_t nb) { return (6 * nb + 1) * 8 + align16(nb * 4) + 64; }
  size_t need_in(request const& r) const { return align16(r.in_bytes); }
  size_t need_out(request const& r) const {
    return encode_ ? align16(rpp_worst_case_bytes(&cfg_, r.n_samples)) + 16 : align16(r.out_cap);
  }
  bool fits(batch const* b, request const& r) const {
    const size_t nb = b->reqs.size() + 1;
    return nb <= kMaxBatchBlocks && b->in_fill + need_in(r) + arrays_in(nb) <= b->in_cap &&
           b->out_fill + need_out(r) + arrays_out(nb) <= b->out_cap;
  }

  // A slot in the open batch for r (lk held); opens a batch when there is
  // none with room, waiting while g_max_active + kSpareBatches are alive.
  batch* reserve(std::unique_lock<std::mutex>& lk, request& r) {
    for (;;) {
      batch* b = open_;
      if (b && fits(b, r)) break;
      if (b && b->reqs.empty()) discard(b);  // (a spare sized for another request)
      else if (b) close(b);                  // full: it goes out as it is
      if (alive_ < g_max_active.load(std::memory_order_relaxed) + kSpareBatches) {
        open_batch(lk, r);
        continue;
      }
      res_cv_.wait(lk);
    }
    batch* b = open_;
    r.in_off = b->in_fill;
    r.out_off = b->out_fill;
    r.pin_in = b->pin_in + r.in_off;
    b->in_fill += need_in(r);
    b->out_fill += need_out(r);
    b->total_samples += r.n_samples;
    b->max_samples = std::max<uint64_t>(b->max_samples, r.n_samples);
    b->reqs.push_back(&r);
    return b;
  }

  void open_batch(std::unique_lock<std::mutex>& lk, request const& r) {
    ++alive_;  // (counted while the context comes up unlocked)
    lk.unlock();
    device_ctx* c = nullptr;
    auto* b = new batch;
    b->t_open = now_ns();
    try {
      const size_t big = std::max(need_in(r), need_out(r));
      const size_t join = need_out(r) > kBatchOut / 4 || need_in(r) > kBatchIn / 4
                              ? std::clamp<size_t>(kLargeJoinBudget / big, 1, kLargeJoin)
                              : 1;
      b->join = join;
      b->in_cap = std::max(kBatchIn, join * need_in(r) + arrays_in(join));
      b->out_cap = std::max(kBatchOut, join * need_out(r) + arrays_out(join));
      c = ctx_pool::get().acquire(dev_, encode_ ? 0 : 1, b->in_cap, b->out_cap);
      device_guard g{dev_};
      b->pin_in = c->pin_in(b->in_cap);
      b->pin_out = c->pin_out(b->out_cap);
      b->ctx = c;
    } catch (...) {
      if (c) ctx_pool::get().release(c);
      delete b;
      lk.lock();
      --alive_;
      res_cv_.notify_all();
      throw;
    }
    lk.lock();
    if (open_) spare_.push_back(b);  // another caller opened one meanwhile: keep ours for later
    else open_ = b;
  }

  // (lk held) an open batch that nobody joined and that is too small for the
  // request at hand
  void discard(batch* b) {
    if (open_ == b) open_ = nullptr;
    discarded_.push_back(b->ctx);  // (returned to the pool once the lock is dropped)
    delete b;
    --alive_;
  }

  // (lk held) no more requests join b
  void close(batch* b) {
    b->closed = true;
    b->t_close = now_ns();
    b->inflight_at_close = inflight_;
    ++inflight_;
    if (open_ == b) {
      open_ = nullptr;
      if (!spare_.empty()) {
        open_ = spare_.back();
        spare_.pop_back();
      }
    }
    if (b->staged == b->reqs.size()) make_ready(b);
  }

  // (lk held) closed and every input copied in: the driver launches it
  // (once the queue is stopping, nothing more is launched)
  void make_ready(batch* b) {
    b->t_ready = now_ns();
    if (stopping_) {
      fail(b, "ricepp_amd: facade shut down");
      return;
    }
    ready_.push_back(b);
    drv_cv_.notify_one();
  }

  // (lk held) a caller leaves run()
  void leave(std::unique_lock<std::mutex>&) {
    if (--active_ == 0 && stopping_) quiet_cv_.notify_all();
  }

  // The driver thread: launches ready batches (the waiter completes them).
  void drive() {
    (void)hipSetDevice(dev_);
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      drv_cv_.wait(lk, [&] { return !ready_.empty() || stopping_; });
      if (stopping_) {
        while (!ready_.empty()) {
          batch* b = ready_.front();
          ready_.pop_front();
          fail(b, "ricepp_amd: facade shut down");
        }
        driver_done_ = true;
        wait_cv_.notify_all();
        return;
      }
      batch* b = ready_.front();
      ready_.pop_front();
      b->t_launch = now_ns();
      lk.unlock();
      std::string err;
      try {
        hip_check(hipEventRecord(b->ctx->start_event(), b->ctx->stream()), "hipEventRecord");
        if (encode_) launch_encode(*b);
        else launch_decode(*b);
        hip_check(hipEventRecord(b->ctx->event(), b->ctx->stream()), "hipEventRecord");
      } catch (std::exception const& e) {
        err = e.what();
        // part of the batch may be on the stream already (copies, kernels
        // writing the mapped pinned output): let it finish before the
        // callers are released and the buffers reused (a stream in error
        // makes release() destroy the context instead of pooling it)
        (void)b->ctx->drain();
      }
      lk.lock();
      if (err.empty()) {
        flight_.push_back(b);
        wait_cv_.notify_one();
      } else {
        fail(b, err);
      }
    }
  }

  // The waiter thread: blocks on the end event of the oldest batch in flight,
  // then also takes the later ones (other streams) that have finished, and
  // publishes their results.  Only this thread removes batches from flight_.
  void wait_loop() {
    (void)hipSetDevice(dev_);
    std::unique_lock<std::mutex> lk(mu_);
    std::vector<batch*> cand;
    std::vector<std::pair<batch*, hipError_t>> fin;
    for (;;) {
      wait_cv_.wait(lk, [&] { return !flight_.empty() || (stopping_ && driver_done_); });
      if (flight_.empty()) return;  // (stopping, and the driver launches nothing more)
      cand.assign(flight_.begin(), flight_.end());
      lk.unlock();
      fin.clear();
      for (size_t i = 0; i < cand.size(); ++i) {
        batch* b = cand[i];
        // the oldest: wait for it; the others: only if already done
        const hipError_t e = i == 0 ? hipEventSynchronize(b->ctx->event()) : hipEventQuery(b->ctx->event());
        if (e == hipErrorNotReady) continue;
        if (e == hipSuccess) {
          float ms = 0.f;
          if (hipEventElapsedTime(&ms, b->ctx->start_event(), b->ctx->event()) == hipSuccess)
            g_device_event_ns.fetch_add(static_cast<uint64_t>(double(ms) * 1e6), std::memory_order_relaxed);
        } else {
          (void)b->ctx->drain();
        }
        fin.emplace_back(b, e);
      }
      lk.lock();
      for (auto [b, e] : fin) {
        flight_.erase(std::find(flight_.begin(), flight_.end(), b));
        if (e != hipSuccess) {
          fail(b, std::string("ricepp_amd: hipEventSynchronize: ") + hipGetErrorString(e));
          continue;
        }
        if (encode_) results_encode(*b);
        else results_decode(*b);
        complete(b);
      }
    }
  }

  void fail(batch* b, std::string const& what) {
    for (request* q : b->reqs) {
      q->status = RPP_HIP_ERROR;
      q->error = what;
      q->result_bytes = 0;
    }
    complete(b);
  }

  // (lk held) every caller of b gets its result; a batch waiting for a free
  // device slot may close now
  void complete(batch* b) {
    b->t_done = now_ns();
    if (!b->t_launch) b->t_launch = b->t_done;  // (failed before its launch)
    --inflight_;
    g_stage_ns.fetch_add(b->t_launch - b->t_close, std::memory_order_relaxed);
    g_device_ns.fetch_add(b->t_done - b->t_launch, std::memory_order_relaxed);
    b->done.store(1, std::memory_order_release);
    b->done.notify_all();
    if (open_ && !open_->reqs.empty() && inflight_ < g_max_active.load(std::memory_order_relaxed)) close(open_);
  }

  // (lk held) the last caller has copied its result out; returns the
  // context, for the caller to pool once it has dropped the lock
  device_ctx* release(batch* b) {
    const uint64_t t_release = now_ns();
    g_finish_ns.fetch_add(t_release - b->t_done, std::memory_order_relaxed);
    if (g_trace_on.load(std::memory_order_relaxed)) {
      std::lock_guard<std::mutex> tl(g_trace_mu);
      g_trace.push_back(facade_batch_record{encode_, (uint32_t)b->reqs.size(), b->in_fill, b->out_fill,
                                            b->inflight_at_close, b->t_open, b->t_close, b->t_ready, b->t_launch,
                                            b->t_done, t_release});
    }
    device_ctx* c = b->ctx;
    delete b;
    --alive_;
    res_cv_.notify_all();
    return c;
  }

  // device: [in][u64 in_off | n | out_off | out_bytes | dst_off | total][i32 status][out slots]
  // pinned in: [in][u64 in_off | n | out_off]   (one H2D copy)
  // pinned out: [packed bytes][u64 out_bytes | dst_off | total][i32 status]
  // The pack kernel writes the encoded bytes straight into the mapped pinned
  // output; the sizes and statuses follow in one small copy.  (The samples
  // are copied in rather than read over PCIe by the encode kernel: reading
  // them in place measured 1.6x slower for 1 MiB blocks and no faster for
  // 64 KiB ones, profiles/r03_facade_bench.jsonl.)
  // RICEPP_AMD_DEBUG_FACADE: 1 prints failed blocks, 2 also checks each
  // request's staged input against its source at launch and at completion,
  // 3 also reads the device copy of the inputs back after the launch
  static int debug_level() {
    static const int v = [] {
      const char* e = std::getenv("RICEPP_AMD_DEBUG_FACADE");
      return e ? std::max(1, std::atoi(e)) : 0;
    }();
    return v;
  }
  void check_staged(batch& b, const char* when) {
    for (size_t i = 0; i < b.reqs.size(); ++i) {
      request* q = b.reqs[i];
      if (q->in_bytes && std::memcmp(q->pin_in, q->in, q->in_bytes) != 0) {
        size_t k = 0;
        while (q->pin_in[k] == q->in[k]) ++k;
        std::fprintf(stderr, "ricepp_amd facade: %s: batch %p req %zu/%zu staged input differs at byte %zu of %zu\n",
                     when, (void*)&b, i, b.reqs.size(), k, q->in_bytes);
      }
    }
  }
  // Device buffers and workspace are asked for at the batch's capacity (its
  // pinned staging, `join` requests of its largest one), not at its fill, so
  // that a context grows them once, on its first batch of a size class: a
  // later, fuller batch regrowing them (hipFree synchronises the device) put
  // a 4-7 ms stall into the first timed 16 MiB run (profiles/r06_facade_16m.jsonl)
  static size_t device_capacity(batch const& b) { return b.in_cap + b.out_cap; }
  uint64_t workspace_capacity(batch const& b, bool encode) const {
    if (b.join <= b.reqs.size()) return 0;
    const uint64_t total = b.join * b.max_samples;
    const auto j = static_cast<uint32_t>(b.join);
    return encode ? rpp_encode_workspace_bytes(&cfg_, total, b.max_samples, j)
                  : rpp_decode_workspace_bytes(&cfg_, total, b.max_samples, j);
  }
  void launch_encode(batch& b) {
    device_ctx& ctx = *b.ctx;
    const size_t nb = b.reqs.size();
    const size_t in_total = b.in_fill, out_total = b.out_fill;
    if (debug_level() >= 2) check_staged(b, "encode launch");
    const size_t arr = (6 * nb + 1) * 8 + align16(nb * 4);
    auto* h64 = reinterpret_cast<uint64_t*>(b.pin_in + in_total);
    for (size_t i = 0; i < nb; ++i) {
      h64[i] = b.reqs[i]->in_off / 2;
      h64[nb + i] = b.reqs[i]->n_samples;
      h64[2 * nb + i] = b.reqs[i]->out_off;
    }
    uint8_t* d = ctx.dev(std::max(in_total + arr + out_total, device_capacity(b)) + 64);
    const uint64_t ws_bytes =
        rpp_encode_workspace_bytes(&cfg_, b.total_samples, b.max_samples, static_cast<uint32_t>(nb));
    uint8_t* ws = ws_bytes ? ctx.workspace(std::max(ws_bytes, workspace_capacity(b, true))) : nullptr;
    uint8_t* pout_dev = ctx.device_view(b.pin_out);
    auto* d64 = reinterpret_cast<uint64_t*>(d + in_total);
    auto* dst = reinterpret_cast<int32_t*>(d + in_total + (6 * nb + 1) * 8);
    uint8_t* dslots = d + in_total + arr;
    hipStream_t s = ctx.stream();
    hip_check(hipMemcpyAsync(d, b.pin_in, in_total + 3 * nb * 8, hipMemcpyHostToDevice, s), "H2D encode input");
    maybe_fail_launch();
    int st = rpp_encode_batch_ws(&cfg_, reinterpret_cast<uint16_t const*>(d), d64, d64 + nb, static_cast<uint32_t>(nb),
                                 dslots, d64 + 2 * nb, d64 + 3 * nb, dst, b.total_samples, b.max_samples, ws, ws_bytes,
                                 s);
    if (st != RPP_OK) throw_status(st);
    if (debug_level() >= 3) {
      std::vector<uint8_t> back(in_total);
      hip_check(hipMemcpyAsync(back.data(), d, in_total, hipMemcpyDeviceToHost, s), "debug D2H");
      ctx.sync();
      for (size_t i = 0; i < nb; ++i) {
        request* q = b.reqs[i];
        if (q->in_bytes && std::memcmp(back.data() + q->in_off, q->in, q->in_bytes) != 0)
          std::fprintf(stderr, "ricepp_amd facade: device copy of req %zu/%zu differs\n", i, nb);
      }
    }
    b.packed = out_total <= g_pack_max.load(std::memory_order_relaxed);
    if (b.packed) {
      st = rpp_pack_batch(dslots, d64 + 2 * nb, d64 + 3 * nb, static_cast<uint32_t>(nb), pout_dev, d64 + 4 * nb,
                          d64 + 5 * nb, s);
      if (st != RPP_OK) throw_status(st);
    } else {
      // long blocks: the slots as they are, by one DMA copy (kernel writes
      // into mapped host memory ran at ~3.5 GB/s for tens of MiB, the copy
      // engine at the PCIe rate; the slots' unused tails cross too)
      hip_check(hipMemcpyAsync(b.pin_out, dslots, out_total, hipMemcpyDeviceToHost, s), "D2H encode slots");
    }
    hip_check(hipMemcpyAsync(b.pin_out + out_total, d64 + 3 * nb, arr - 3 * nb * 8, hipMemcpyDeviceToHost, s),
              "D2H encode sizes");
    g_enc_launches.fetch_add(1, std::memory_order_relaxed);
    g_enc_blocks.fetch_add(nb, std::memory_order_relaxed);
  }
  void results_encode(batch& b) {
    const size_t nb = b.reqs.size();
    if (debug_level() >= 2) check_staged(b, "encode done");
    auto const* r64 = reinterpret_cast<uint64_t const*>(b.pin_out + b.out_fill);  // out_bytes | dst_off | total
    auto const* hst = reinterpret_cast<int32_t const*>(b.pin_out + b.out_fill + (3 * nb + 1) * 8);
    for (size_t i = 0; i < nb; ++i) {
      request* q = b.reqs[i];
      q->status = hst[i];
      q->result_bytes = hst[i] == RPP_OK ? r64[i] : 0;
      q->pin_out = b.pin_out + (b.packed ? r64[nb + i] : q->out_off);
      if (q->status == RPP_OK && q->result_bytes > q->out_cap) q->status = RPP_OUTPUT_TOO_SMALL;
      if (q->status != RPP_OK && debug_level())
        std::fprintf(stderr, "ricepp_amd facade: encode batch nb=%zu total=%llu max=%llu in_fill=%zu out_fill=%zu "
                     "packed=%d: block %zu n=%llu in_off=%zu out_off=%zu status=%d\n", nb,
                     (unsigned long long)b.total_samples, (unsigned long long)b.max_samples, b.in_fill, b.out_fill,
                     (int)b.packed, i, (unsigned long long)q->n_samples, q->in_off, q->out_off, q->status);
    }
  }

  // device: [in][u64 in_off | in_bytes | out_off | n][out samples][i32 status]
  // pinned in: [in][u64 in_off | in_bytes | out_off | n]   (one H2D copy)
  // pinned out: [out samples][i32 status]                  (one D2H copy)
  // (batches of short streams only: no device buffers, the kernel works on
  // the pinned buffers themselves)
  void launch_decode(batch& b) {
    device_ctx& ctx = *b.ctx;
    const size_t nb = b.reqs.size();
    const size_t in_total = b.in_fill, out_total = b.out_fill;
    auto* h64 = reinterpret_cast<uint64_t*>(b.pin_in + in_total);
    for (size_t i = 0; i < nb; ++i) {
      h64[i] = b.reqs[i]->in_off;
      h64[nb + i] = b.reqs[i]->in_bytes;
      h64[2 * nb + i] = b.reqs[i]->out_off / 2;
      h64[3 * nb + i] = b.reqs[i]->n_samples;
    }
    const size_t st_bytes = align16(nb * 4);
    // long blocks (16 MiB DwarFS blocks) are parsed in segments by several waves
    const uint64_t ws_bytes =
        rpp_decode_workspace_bytes(&cfg_, b.total_samples, b.max_samples, static_cast<uint32_t>(nb));
    hipStream_t s = ctx.stream();
    if (ws_bytes == 0) {
      // every stream is decoded by one wave, which reads its compressed bytes
      // once (through its LDS ring, prefetched far ahead) and writes each
      // sample once: straight from and to the mapped pinned buffers, no
      // copies (a batch of short streams is latency-bound, and copies on two
      // streams at once do not overlap with the kernels)
      uint8_t* din = ctx.device_view(b.pin_in);
      uint8_t* dout = ctx.device_view(b.pin_out);
      auto* d64 = reinterpret_cast<uint64_t*>(din + in_total);
      int st = rpp_decode_batch_ws(&cfg_, din, d64, d64 + nb, static_cast<uint32_t>(nb),
                                   reinterpret_cast<uint16_t*>(dout), d64 + 2 * nb, d64 + 3 * nb,
                                   reinterpret_cast<int32_t*>(dout + out_total), b.total_samples, b.max_samples,
                                   nullptr, 0, s);
      if (st != RPP_OK) throw_status(st);
      maybe_fail_launch();
      g_dec_launches.fetch_add(1, std::memory_order_relaxed);
      g_dec_blocks.fetch_add(nb, std::memory_order_relaxed);
      return;
    }
    uint8_t* d = ctx.dev(std::max(in_total + 4 * nb * 8 + out_total + st_bytes, device_capacity(b)) + 64);
    uint8_t* ws = ctx.workspace(std::max(ws_bytes, workspace_capacity(b, false)));
    auto* d64 = reinterpret_cast<uint64_t*>(d + in_total);
    uint8_t* dout = d + in_total + 4 * nb * 8;
    auto* dst = reinterpret_cast<int32_t*>(dout + out_total);
    hip_check(hipMemcpyAsync(d, b.pin_in, in_total + 4 * nb * 8, hipMemcpyHostToDevice, s), "H2D decode input");
    maybe_fail_launch();
    int st = rpp_decode_batch_ws(&cfg_, d, d64, d64 + nb, static_cast<uint32_t>(nb), reinterpret_cast<uint16_t*>(dout),
                                 d64 + 2 * nb, d64 + 3 * nb, dst, b.total_samples, b.max_samples, ws, ws_bytes, s);
    if (st != RPP_OK) throw_status(st);
    hip_check(hipMemcpyAsync(b.pin_out, dout, out_total + st_bytes, hipMemcpyDeviceToHost, s), "D2H decoded");
    g_dec_launches.fetch_add(1, std::memory_order_relaxed);
    g_dec_blocks.fetch_add(nb, std::memory_order_relaxed);
  }
  void results_decode(batch& b) {
    auto const* hst = reinterpret_cast<int32_t const*>(b.pin_out + b.out_fill);
    for (size_t i = 0; i < b.reqs.size(); ++i) {
      request* q = b.reqs[i];
      q->status = hst[i];
      q->result_bytes = hst[i] == RPP_OK ? q->out_cap : 0;
      q->pin_out = b.pin_out + q->out_off;
    }
  }

  int dev_;
  rpp_config cfg_;
  bool encode_;
  std::mutex mu_;
  std::condition_variable res_cv_;  // callers waiting for a batch with room
  std::condition_variable drv_cv_;  // the driver, waiting for a ready batch
  std::condition_variable wait_cv_;  // the waiter, waiting for a batch in flight
  std::condition_variable quiet_cv_;  // shutdown, waiting for callers to leave run()
  batch* open_ = nullptr;           // the batch taking new requests
  std::vector<batch*> spare_;       // opened concurrently, not yet taking requests
  std::deque<batch*> ready_;        // closed and staged, to be launched
  std::deque<batch*> flight_;       // launched, in launch order
  std::vector<device_ctx*> discarded_;  // contexts of discarded batches, to pool unlocked
  int inflight_ = 0;                // closed, not yet completed
  int alive_ = 0;
  int active_ = 0;                  // callers inside run()
  bool stopping_ = false, driver_done_ = false;
  std::thread driver_, waiter_;
};

// The queues (intentionally never destroyed: their threads are stopped by
// shutdown_facade(), which std::atexit runs before the HIP runtime's own
// teardown -- it is registered after the runtime has come up).
struct queue_registry {
  std::mutex mu;
  std::map<std::tuple<int, uint32_t, uint32_t, uint32_t, uint32_t, bool>, batch_queue*> queues;
};
queue_registry& registry() {
  static auto* r = new queue_registry;
  return *r;
}

void shutdown_all() {
  g_shutdown.store(true, std::memory_order_release);
  std::vector<batch_queue*> qs;
  {
    std::lock_guard<std::mutex> lk(registry().mu);
    for (auto& [k, q] : registry().queues) qs.push_back(q);
  }
  for (batch_queue* q : qs) q->shutdown();
}

batch_queue& queue_for(int dev, rpp_config const& c, bool encode) {
  auto& reg = registry();
  std::lock_guard<std::mutex> lk(reg.mu);
  if (g_shutdown.load(std::memory_order_acquire)) throw std::runtime_error("ricepp_amd: facade shut down");
  static const bool registered = [] { return std::atexit(shutdown_all) == 0; }();
  (void)registered;
  auto key = std::make_tuple(dev, c.block_size, c.component_stream_count, c.big_endian, c.unused_lsb_count, encode);
  auto it = reg.queues.find(key);
  if (it == reg.queues.end()) it = reg.queues.emplace(key, new batch_queue(dev, c, encode)).first;
  return *it->second;
}

// Runs one request through its queue (the calling thread may become the
// leader of a batch that contains it).
void submit(batch_queue& q, request& r) {
  q.run(r);
  if (r.status == RPP_HIP_ERROR) throw std::runtime_error(r.error.empty() ? "ricepp_amd: HIP error" : r.error);
  if (r.status != RPP_OK) throw_status(r.status);
}

class encoder_impl final : public encoder_interface<uint16_t> {
 public:
  encoder_impl(rpp_config c, int dev) : cfg_{c}, q_{queue_for(dev, c, true)} {}

  size_t worst_case_encoded_bytes(size_t n) const override { return rpp_worst_case_bytes(&cfg_, n); }
  size_t worst_case_encoded_bytes(std::span<uint16_t const> in) const override {
    return worst_case_encoded_bytes(in.size());
  }

  std::vector<uint8_t> encode(std::span<uint16_t const> input) const override {
    std::vector<uint8_t> out(worst_case_encoded_bytes(input.size()));
    auto used = encode(std::span<uint8_t>{out}, input);
    out.resize(used.size());
    return out;
  }

  // ricepp_cpuspecific.cpp:101-108: output must hold the worst case
  std::span<uint8_t> encode(std::span<uint8_t> output, std::span<uint16_t const> input) const override {
    if (output.size() < worst_case_encoded_bytes(input.size()))
      throw std::length_error("ricepp_amd: output smaller than worst_case_encoded_bytes");
    if (input.size() % cfg_.component_stream_count) throw_status(RPP_INVALID_ARGUMENT);
    request r{reinterpret_cast<uint8_t const*>(input.data()), input.size_bytes(), output.data(), output.size(),
              input.size()};
    submit(q_, r);
    return output.subspan(0, r.result_bytes);
  }

 private:
  rpp_config cfg_;
  batch_queue& q_;
};

class decoder_impl final : public decoder_interface<uint16_t> {
 public:
  decoder_impl(rpp_config c, int dev) : cfg_{c}, q_{queue_for(dev, c, false)} {}

  // ricepp_cpuspecific.cpp:127-144: decodes exactly output.size() samples
  void decode(std::span<uint16_t> output, std::span<uint8_t const> input) const override {
    if (output.size() % cfg_.component_stream_count) throw_status(RPP_INVALID_ARGUMENT);
    request r{input.data(), input.size(), reinterpret_cast<uint8_t*>(output.data()), output.size_bytes(),
              output.size()};
    submit(q_, r);
  }

 private:
  rpp_config cfg_;
  batch_queue& q_;
};

// ---- minimal JSON for the flat metadata objects of the plugin ----
// (the reference uses nlohmann::json; only string and integer members occur)
std::map<std::string, std::string> parse_flat_json(std::string const& s) {
  std::map<std::string, std::string> m;
  size_t i = 0;
  auto skip = [&] {
    while (i < s.size() && std::isspace(static_cast<unsigned char>(s[i]))) ++i;
  };
  auto str = [&]() -> std::string {
    std::string r;
    if (i >= s.size() || s[i] != '"') throw std::runtime_error("ricepp_amd: malformed metadata JSON");
    for (++i; i < s.size() && s[i] != '"'; ++i) {
      if (s[i] == '\\' && i + 1 < s.size()) ++i;
      r += s[i];
    }
    ++i;
    return r;
  };
  skip();
  if (i >= s.size() || s[i] != '{') throw std::runtime_error("ricepp_amd: malformed metadata JSON");
  ++i;
  for (;;) {
    skip();
    if (i >= s.size()) throw std::runtime_error("ricepp_amd: malformed metadata JSON");
    if (s[i] == '}') break;
    std::string k = str();
    skip();
    if (i >= s.size() || s[i] != ':') throw std::runtime_error("ricepp_amd: malformed metadata JSON");
    ++i;
    skip();
    std::string v;
    if (i < s.size() && s[i] == '"') {
      v = "\"" + str();
    } else {
      while (i < s.size() && s[i] != ',' && s[i] != '}' && !std::isspace(static_cast<unsigned char>(s[i]))) v += s[i++];
    }
    m[k] = v;
    skip();
    if (i < s.size() && s[i] == ',') ++i;
  }
  return m;
}

int json_int(std::map<std::string, std::string> const& m, char const* key) {
  auto it = m.find(key);
  if (it == m.end() || it->second.empty() || it->second[0] == '"')
    throw std::runtime_error(std::string("ricepp_amd: metadata lacks integer '") + key + "'");
  int v = 0;
  auto r = std::from_chars(it->second.data(), it->second.data() + it->second.size(), v);
  if (r.ec != std::errc{}) throw std::runtime_error(std::string("ricepp_amd: bad integer '") + key + "'");
  return v;
}

std::string json_str(std::map<std::string, std::string> const& m, char const* key) {
  auto it = m.find(key);
  if (it == m.end() || it->second.empty() || it->second[0] != '"')
    throw std::runtime_error(std::string("ricepp_amd: metadata lacks string '") + key + "'");
  return it->second.substr(1);
}

constexpr uint32_t kRiceppVersion = 1;  // src/compression/ricepp.cpp:55

}  // namespace

template <>
std::unique_ptr<encoder_interface<uint16_t>> create_encoder<uint16_t>(codec_config const& config) {
  rpp_config c = to_rpp(config);
  if (rpp_check_config(&c) != RPP_OK) throw std::runtime_error("Unsupported configuration");
  return std::make_unique<encoder_impl>(c, current_device());
}

template <>
std::unique_ptr<decoder_interface<uint16_t>> create_decoder<uint16_t>(codec_config const& config) {
  rpp_config c = to_rpp(config);
  if (rpp_check_config(&c) != RPP_OK) throw std::runtime_error("Unsupported configuration");
  return std::make_unique<decoder_impl>(c, current_device());
}

void inject_context_failures(uint32_t n) { g_ctx_faults.store(n); }

void inject_launch_failures(uint32_t n) { g_launch_faults.store(n); }

void set_facade_pipeline_depth(int batches) { g_max_active.store(std::max(1, std::min(batches, 16))); }
void set_facade_pack_limit(size_t bytes) { g_pack_max.store(bytes); }
void set_facade_large_min_fill(int requests) { g_large_min_fill.store(std::max(1, requests)); }

facade_stats get_facade_stats() {
  return facade_stats{g_enc_launches.load(), g_enc_blocks.load(), g_dec_launches.load(), g_dec_blocks.load(),
                      g_ctx_created.load(),  g_stage_ns.load(),   g_device_ns.load(),    g_finish_ns.load(),
                      g_device_event_ns.load(), g_buffer_grows.load(), g_buffer_grow_ns.load()};
}

void shutdown_facade() { shutdown_all(); }

void set_facade_trace(bool on) { g_trace_on.store(on); }
std::vector<facade_batch_record> take_facade_trace() {
  std::lock_guard<std::mutex> tl(g_trace_mu);
  std::vector<facade_batch_record> out;
  out.swap(g_trace);
  return out;
}

// ---- block_compressor (src/compression/ricepp.cpp:57-182, 272-296) ----

block_compressor::block_compressor(size_t block_size) : block_size_{block_size} {}

std::unique_ptr<block_compressor> block_compressor::create(std::string const& spec) {
  // "ricepp" or "ricepp:block_size=N" (option_map, default 128, :280); like
  // the reference's factory, the value is not range-checked here
  size_t bs = 128;
  std::string name = spec.substr(0, spec.find(':'));
  if (name != "ricepp") throw std::runtime_error("unknown compression: " + name);
  if (auto c = spec.find(':'); c != std::string::npos) {
    std::string opts = spec.substr(c + 1);
    size_t p = 0;
    while (p < opts.size()) {
      size_t e = opts.find(',', p);
      std::string kv = opts.substr(p, e == std::string::npos ? std::string::npos : e - p);
      auto eq = kv.find('=');
      if (kv.substr(0, eq) != "block_size" || eq == std::string::npos)
        throw std::runtime_error("invalid option(s) for ricepp: " + kv);
      bs = std::stoul(kv.substr(eq + 1));
      if (e == std::string::npos) break;
      p = e + 1;
    }
  }
  return std::make_unique<block_compressor>(bs);
}

std::unique_ptr<block_compressor> block_compressor::clone() const {
  return std::make_unique<block_compressor>(*this);
}

std::string block_compressor::describe() const { return "ricepp [block_size=" + std::to_string(block_size_) + "]"; }

std::string block_compressor::metadata_requirements() const {
  // ricepp.cpp:150-159 (nlohmann::json dump: keys sorted)
  return R"({"bytes_per_sample":["set",[2]],"component_count":["range",1,2],)"
         R"("endianness":["set",["big","little"]],"unused_lsb_count":["range",0,8]})";
}

size_t block_compressor::compression_granularity(std::string const& metadata) const {
  auto m = parse_flat_json(metadata);  // ricepp.cpp:161-173
  return static_cast<size_t>(json_int(m, "component_count") * json_int(m, "bytes_per_sample"));
}

std::vector<uint8_t> block_compressor::compress(std::span<uint8_t const> data, std::string const* metadata) const {
  if (!metadata) throw std::runtime_error("internal error: ricepp compression requires metadata");  // :70-73
  auto meta = parse_flat_json(*metadata);
  auto endianness = json_str(meta, "endianness");
  int component_count = json_int(meta, "component_count");
  int unused_lsb_count = json_int(meta, "unused_lsb_count");
  int bytes_per_sample = json_int(meta, "bytes_per_sample");
  if (bytes_per_sample != 2 || unused_lsb_count < 0 || unused_lsb_count > 8 || component_count < 1 ||
      component_count > 2)
    throw std::runtime_error("ricepp_amd: metadata out of range");  // asserts at :82-84
  if (data.size() % static_cast<size_t>(component_count * bytes_per_sample))  // :86-91
    throw std::runtime_error("unexpected data configuration: " + std::to_string(data.size()) +
                             " bytes to compress, " + std::to_string(component_count) + " components, " +
                             std::to_string(bytes_per_sample) + " bytes per sample");
  auto const byteorder = endianness == "big" ? std::endian::big : std::endian::little;
  // :97-102 -- throws "Unsupported configuration" for an unsupported block size
  auto enc = create_encoder<uint16_t>({
      .block_size = block_size_,
      .component_stream_count = static_cast<size_t>(component_count),
      .byteorder = byteorder,
      .unused_lsb_count = static_cast<unsigned>(unused_lsb_count),
  });
  rpp_frame f{data.size(), static_cast<uint32_t>(block_size_), static_cast<uint32_t>(component_count),
              static_cast<uint32_t>(bytes_per_sample), static_cast<uint32_t>(unused_lsb_count),
              byteorder == std::endian::big ? 1u : 0u, kRiceppVersion};
  std::vector<uint8_t> out(64);
  size_t hdr = rpp_frame_header(&f, out.data());
  size_t n = data.size() / 2;
  out.resize(hdr + enc->worst_case_encoded_bytes(n));
  // (the samples are read in place: the staging copy handles any alignment)
  std::span<uint16_t const> samples{reinterpret_cast<uint16_t const*>(data.data()), n};
  auto used = enc->encode(std::span<uint8_t>{out}.subspan(hdr), samples);
  out.resize(hdr + used.size());
  out.shrink_to_fit();
  return out;
}

// ---- block_decompressor (src/compression/ricepp.cpp:184-255) ----

block_decompressor::block_decompressor(std::span<uint8_t const> data) {
  long h = rpp_parse_frame(data.data(), data.size(), &frame_);
  if (h < 0) throw std::runtime_error("ricepp_amd: malformed ricepp block header");
  data_ = data.subspan(static_cast<size_t>(h));
  if (frame_.ricepp_version > kRiceppVersion)  // :243-247
    throw std::runtime_error("[RICEPP] unsupported version: " + std::to_string(frame_.ricepp_version));
  decoder_ = create_decoder<uint16_t>({
      .block_size = frame_.block_size,
      .component_stream_count = frame_.component_count,
      .byteorder = frame_.big_endian ? std::endian::big : std::endian::little,
      .unused_lsb_count = frame_.unused_lsb_count,
  });
  if (frame_.bytes_per_sample != 2)  // :196-200
    throw std::runtime_error("[RICEPP] unsupported bytes per sample: " + std::to_string(frame_.bytes_per_sample));
}

std::optional<std::string> block_decompressor::metadata() const {
  // :203-212 (nlohmann::json dump: keys sorted)
  return std::string(R"({"bytes_per_sample":)") + std::to_string(frame_.bytes_per_sample) +
         R"(,"component_count":)" + std::to_string(frame_.component_count) + R"(,"endianness":")" +
         (frame_.big_endian ? "big" : "little") + R"(","unused_lsb_count":)" +
         std::to_string(frame_.unused_lsb_count) + "}";
}

void block_decompressor::start_decompression(std::vector<uint8_t>* target) {
  target_ = target;
  target_->reserve(frame_.uncompressed_bytes);  // src/compression/base.cpp:37-51
}

bool block_decompressor::decompress_frame(size_t) {
  if (!target_) throw std::runtime_error("decompression not started");  // :216
  if (!decoder_) return false;
  target_->resize(frame_.uncompressed_bytes);
  std::span<uint16_t> out{reinterpret_cast<uint16_t*>(target_->data()), target_->size() / 2};
  decoder_->decode(out, data_);
  decoder_.reset();
  return true;
}

std::vector<uint8_t> block_decompressor::decompress(std::span<uint8_t const> data) {
  block_decompressor d{data};
  std::vector<uint8_t> out;
  d.start_decompression(&out);
  d.decompress_frame(d.uncompressed_size());
  return out;
}

// ---- pcm_sample_transformer (src/pcm_sample_transformer.cpp:372-377) ----

pcm_sample_transformer::pcm_sample_transformer(pcm_sample_endianness end, pcm_sample_signedness sig,
                                               pcm_sample_padding pad, int bytes, int bits) {
  fmt_.big_endian = end == pcm_sample_endianness::Big ? 1u : 0u;
  fmt_.is_signed = sig == pcm_sample_signedness::Signed ? 1u : 0u;
  fmt_.lsb_padded = pad == pcm_sample_padding::Lsb ? 1u : 0u;
  fmt_.bytes = bytes < 0 ? 0u : static_cast<uint32_t>(bytes);
  fmt_.bits = bits < 0 ? 0u : static_cast<uint32_t>(bits);
  const int st = rpp_pcm_check_format(&fmt_);
  if (st == RPP_UNSUPPORTED_CONFIG || bytes < 1 || bytes > 4)
    throw std::runtime_error("unsupported number of bytes per sample: " + std::to_string(bytes));
  if (st != RPP_OK) throw std::invalid_argument("pcm_sample_transformer: bits outside 1..8*bytes");
  device_ = current_device();
}

pcm_sample_transformer::~pcm_sample_transformer() = default;
pcm_sample_transformer::pcm_sample_transformer(pcm_sample_transformer&&) noexcept = default;
pcm_sample_transformer& pcm_sample_transformer::operator=(pcm_sample_transformer&&) noexcept = default;

void pcm_sample_transformer::unpack(std::span<int32_t> dst, std::span<uint8_t const> src) const {
  if (src.size() != fmt_.bytes * dst.size()) throw std::invalid_argument("pcm unpack: src.size() != bytes * dst.size()");
  if (dst.empty()) return;
  const size_t off_out = align16(src.size());
  device_guard g{device_};
  ctx_lease ctx{device_};
  uint8_t* d = ctx->dev(off_out + dst.size_bytes());
  hipStream_t s = ctx->stream();
  hip_check(hipMemcpyAsync(d, src.data(), src.size(), hipMemcpyHostToDevice, s), "H2D pcm");
  const int st = rpp_pcm_unpack(&fmt_, d, reinterpret_cast<int32_t*>(d + off_out), dst.size(), s);
  if (st != RPP_OK) throw_status(st);
  hip_check(hipMemcpyAsync(dst.data(), d + off_out, dst.size_bytes(), hipMemcpyDeviceToHost, s), "D2H pcm");
  ctx->sync();
}

void pcm_sample_transformer::pack(std::span<uint8_t> dst, std::span<int32_t const> src) const {
  if (dst.size() != fmt_.bytes * src.size()) throw std::invalid_argument("pcm pack: dst.size() != bytes * src.size()");
  if (src.empty()) return;
  const size_t off_out = align16(src.size_bytes());
  device_guard g{device_};
  ctx_lease ctx{device_};
  uint8_t* d = ctx->dev(off_out + dst.size());
  hipStream_t s = ctx->stream();
  hip_check(hipMemcpyAsync(d, src.data(), src.size_bytes(), hipMemcpyHostToDevice, s), "H2D pcm");
  const int st = rpp_pcm_pack(&fmt_, reinterpret_cast<int32_t const*>(d), d + off_out, src.size(), s);
  if (st != RPP_OK) throw_status(st);
  hip_check(hipMemcpyAsync(dst.data(), d + off_out, dst.size(), hipMemcpyDeviceToHost, s), "D2H pcm");
  ctx->sync();
}

// ---- FLAC block codec (src/compression/flac.cpp:215-525) ----

namespace {

constexpr uint32_t kFlacBigEndian = 0x80, kFlacSigned = 0x40, kFlacLsbPadding = 0x20, kFlacBytesMask = 0x03;  // :41-44

char const* status_name(int st) {
  switch (st) {
    case RPP_OK: return "OK";
    case RPP_UNSUPPORTED_CONFIG: return "UNSUPPORTED_CONFIG";
    case RPP_TRUNCATED_INPUT: return "TRUNCATED_INPUT";
    case RPP_INVALID_ARGUMENT: return "INVALID_ARGUMENT";
    case RPP_OUTPUT_TOO_SMALL: return "OUTPUT_TOO_SMALL";
    case RPP_HIP_ERROR: return "HIP_ERROR";
    case RPP_INTERNAL_ERROR: return "INTERNAL_ERROR";
    default: return "UNKNOWN";
  }
}

rpp_pcm_format flac_pcm_format(uint32_t flags, uint32_t bits) {
  rpp_pcm_format f{};
  f.big_endian = flags & kFlacBigEndian ? 1u : 0u;
  f.is_signed = flags & kFlacSigned ? 1u : 0u;
  f.lsb_padded = flags & kFlacLsbPadding ? 1u : 0u;
  f.bytes = (flags & kFlacBytesMask) + 1;
  f.bits = bits;
  return f;
}

}  // namespace

flac_block_compressor::flac_block_compressor(uint32_t level, bool exhaustive) : level_{level}, exhaustive_{exhaustive} {
  if (level_ > 8) throw std::runtime_error("invalid option(s) for flac: level=" + std::to_string(level_));
}

std::unique_ptr<flac_block_compressor> flac_block_compressor::create(std::string const& spec) {
  // option_map over "flac:level=N:exhaustive" (flac.cpp:509-525; options
  // separated by ':' or ',')
  std::string name = spec.substr(0, spec.find(':'));
  if (name != "flac") throw std::runtime_error("unknown compression: " + name);
  uint32_t level = 5;
  bool exhaustive = false;
  if (auto c = spec.find(':'); c != std::string::npos) {
    std::string opts = spec.substr(c + 1);
    size_t p = 0;
    while (p <= opts.size()) {
      size_t e = opts.find_first_of(",:", p);
      std::string kv = opts.substr(p, e == std::string::npos ? std::string::npos : e - p);
      if (!kv.empty()) {
        auto eq = kv.find('=');
        std::string k = kv.substr(0, eq);
        if (k == "level" && eq != std::string::npos) {
          std::string v = kv.substr(eq + 1);
          unsigned long lv = 0;
          auto r = std::from_chars(v.data(), v.data() + v.size(), lv);
          if (r.ec != std::errc{} || r.ptr != v.data() + v.size() || lv > 8)
            throw std::runtime_error("invalid option(s) for flac: " + kv);
          level = static_cast<uint32_t>(lv);
        } else if (k == "exhaustive" && eq == std::string::npos) {
          exhaustive = true;
        } else {
          throw std::runtime_error("invalid option(s) for flac: " + kv);
        }
      }
      if (e == std::string::npos) break;
      p = e + 1;
    }
  }
  return std::make_unique<flac_block_compressor>(level, exhaustive);
}

std::unique_ptr<flac_block_compressor> flac_block_compressor::clone() const {
  return std::make_unique<flac_block_compressor>(*this);
}

std::string flac_block_compressor::describe() const {
  return "flac [level=" + std::to_string(level_) + (exhaustive_ ? ", exhaustive" : "") + "]";
}

std::string flac_block_compressor::metadata_requirements() const {
  // flac.cpp:368-379 (nlohmann::json dump: keys sorted)
  return R"({"bits_per_sample":["range",8,32],"bytes_per_sample":["range",1,4],"endianness":["set",["big","little"]],)"
         R"("number_of_channels":["range",1,8],"padding":["set",["msb","lsb"]],"signedness":["set",["signed","unsigned"]]})";
}

size_t flac_block_compressor::compression_granularity(std::string const& metadata) const {
  auto m = parse_flat_json(metadata);
  return static_cast<size_t>(json_int(m, "number_of_channels") * json_int(m, "bytes_per_sample"));
}

std::vector<uint8_t> flac_block_compressor::compress(std::span<uint8_t const> data, std::string const* metadata) const {
  if (!metadata) throw std::runtime_error("internal error: flac compression requires metadata");  // :229-232
  auto meta = parse_flat_json(*metadata);
  const std::string endianness = json_str(meta, "endianness"), signedness = json_str(meta, "signedness"),
                    padding = json_str(meta, "padding");
  const int channels = json_int(meta, "number_of_channels"), bits = json_int(meta, "bits_per_sample"),
            nbytes = json_int(meta, "bytes_per_sample");
  if (nbytes < 1 || nbytes > 4 || bits < 8 || bits > 32 || channels < 1)  // asserts at :243-245
    throw std::runtime_error("ricepp_amd: flac metadata out of range");
  if (data.size() % static_cast<size_t>(channels * nbytes))  // :247-253
    throw std::runtime_error("unexpected PCM waveform configuration: " + std::to_string(data.size()) +
                             " bytes to compress, " + std::to_string(channels) + " channels, " +
                             std::to_string(nbytes) + " bytes per sample");
  uint32_t flags = static_cast<uint32_t>(nbytes - 1);
  if (endianness == "big") flags |= kFlacBigEndian;
  if (signedness == "signed") flags |= kFlacSigned;
  if (padding == "lsb") flags |= kFlacLsbPadding;
  const uint64_t n = data.size() / static_cast<size_t>(channels * nbytes);  // samples per channel
  rpp_flac_frame f{data.size(), static_cast<uint32_t>(channels), static_cast<uint32_t>(bits), flags};
  std::vector<uint8_t> out(128);
  size_t hdr = rpp_flac_frame_header(&f, out.data());
  hdr += rpp_flac_stream_header(f.num_channels, f.bits_per_sample, n, out.data() + hdr);
  out.resize(hdr);
  if (n == 0) return out;
  // libFLAC's encoder init rejects what it cannot code (:313-317)
  const uint64_t bound = rpp_flac_frame_bound(f.num_channels, f.bits_per_sample);
  if (channels > 8 || bound == 0) throw std::runtime_error("[FLAC] init: unsupported stream shape");
  const rpp_pcm_format pf = flac_pcm_format(flags, f.bits_per_sample);
  const uint64_t nvals = n * static_cast<uint64_t>(channels);
  const uint64_t frames = (n + 4095) / 4096;
  const uint64_t ws_bytes = rpp_flac_encode_workspace_bytes(n, f.num_channels, f.bits_per_sample);
  const size_t off_x = align16(data.size()), off_out = off_x + align16(nvals * 4),
               off_tot = off_out + align16(frames * bound + 64), off_ws = off_tot + 16;
  const int dev = current_device();
  device_guard g{dev};
  ctx_lease ctx{dev};
  uint8_t* d = ctx->dev(off_ws + ws_bytes);
  hipStream_t st = ctx->stream();
  hip_check(hipMemcpyAsync(d, data.data(), data.size(), hipMemcpyHostToDevice, st), "H2D flac pcm");
  int rc = rpp_pcm_unpack(&pf, d, reinterpret_cast<int32_t*>(d + off_x), nvals, st);
  if (rc != RPP_OK) throw std::runtime_error(std::string("[FLAC] failed to process interleaved samples: ") + status_name(rc));
  rc = rpp_flac_encode_ex(reinterpret_cast<int32_t const*>(d + off_x), n, f.num_channels, f.bits_per_sample, level_,
                          exhaustive_ ? 1u : 0u, d + off_out, reinterpret_cast<uint64_t*>(d + off_tot), d + off_ws,
                          ws_bytes, st);
  if (rc != RPP_OK) throw std::runtime_error(std::string("[FLAC] failed to process interleaved samples: ") + status_name(rc));
  uint64_t total = 0;
  hip_check(hipMemcpyAsync(&total, d + off_tot, 8, hipMemcpyDeviceToHost, st), "D2H flac size");
  ctx->sync();
  out.resize(hdr + total);
  hip_check(hipMemcpyAsync(out.data() + hdr, d + off_out, total, hipMemcpyDeviceToHost, st), "D2H flac frames");
  ctx->sync();
  return out;
}

flac_block_decompressor::flac_block_decompressor(std::span<uint8_t const> data) {
  long h = rpp_flac_parse_frame(data.data(), data.size(), &frame_);
  if (h < 0) throw std::runtime_error("ricepp_amd: malformed flac block header");
  auto stream = data.subspan(static_cast<size_t>(h));
  long at = rpp_flac_parse_stream(stream.data(), stream.size(), &info_);
  if (at < 0)  // :410-418
    throw std::runtime_error(std::string("[FLAC] could not initialize decoder: ") + status_name(static_cast<int>(at)));
  frames_ = stream.subspan(static_cast<size_t>(at));
}

std::optional<std::string> flac_block_decompressor::metadata() const {
  // :429-440 (nlohmann::json dump: keys sorted)
  const uint32_t fl = frame_.flags;
  return std::string(R"({"bits_per_sample":)") + std::to_string(frame_.bits_per_sample) +
         R"(,"bytes_per_sample":)" + std::to_string((fl & kFlacBytesMask) + 1) + R"(,"endianness":")" +
         (fl & kFlacBigEndian ? "big" : "little") + R"(","number_of_channels":)" +
         std::to_string(frame_.num_channels) + R"(,"padding":")" + (fl & kFlacLsbPadding ? "lsb" : "msb") +
         R"(","signedness":")" + (fl & kFlacSigned ? "signed" : "unsigned") + "\"}";
}

void flac_block_decompressor::start_decompression(std::vector<uint8_t>* target) {
  target_ = target;
  target_->reserve(frame_.uncompressed_bytes);
}

bool flac_block_decompressor::decompress_frame(size_t) {
  if (!target_) throw std::runtime_error("decompression not started");
  if (done_) return false;
  const uint32_t channels = info_.channels, bits = info_.bits_per_sample;
  const uint32_t nbytes = (frame_.flags & kFlacBytesMask) + 1;
  const uint64_t n = info_.total_samples;
  auto fail = [](std::string const& why) { return std::runtime_error("[FLAC] failed to process frame: " + why); };
  if (n * channels * nbytes != frame_.uncompressed_bytes) throw fail("stream length does not match the block");
  target_->resize(frame_.uncompressed_bytes);
  done_ = true;
  if (n == 0) return true;
  // frames: at most n / min_blocksize + 1; spurious sync codes passing the
  // CRC-8 are rare and retried with room for all.  A block-size range that
  // would size the per-candidate scratch beyond 4x the block's samples is
  // refused (libFLAC and DwarFS's compressor write min == max).
  const uint64_t min_bs = std::max<uint64_t>(16, info_.min_blocksize ? info_.min_blocksize : 16);
  const uint64_t max_bs = info_.max_blocksize ? info_.max_blocksize : 65535;
  uint64_t max_cand = n / min_bs + 65;
  auto too_wide = [&](uint64_t cand) { return cand * max_bs > 4 * n + 128 * max_bs; };
  if (too_wide(max_cand)) throw fail("block size range too wide for the block");
  const rpp_pcm_format pf = flac_pcm_format(frame_.flags, frame_.bits_per_sample);
  const uint64_t nvals = n * channels;
  const int dev = current_device();
  device_guard g{dev};
  ctx_lease ctx{dev};
  hipStream_t st = ctx->stream();
  for (int attempt = 0;; ++attempt) {
    const uint64_t ws_bytes = rpp_flac_decode_workspace_bytes(frames_.size(), channels, bits,
                                                              static_cast<uint32_t>(max_bs),
                                                              static_cast<uint32_t>(max_cand));
    const size_t off_x = align16(frames_.size()), off_pcm = off_x + align16(nvals * 4),
                 off_st = off_pcm + align16(frame_.uncompressed_bytes), off_ws = off_st + 16;
    uint8_t* d = ctx->dev(off_ws + ws_bytes);
    auto* dst = reinterpret_cast<int32_t*>(d + off_st);
    hip_check(hipMemcpyAsync(d, frames_.data(), frames_.size(), hipMemcpyHostToDevice, st), "H2D flac frames");
    hip_check(hipMemsetAsync(dst, 0, 8, st), "hipMemsetAsync");
    int rc = rpp_flac_decode(d, frames_.size(), channels, bits, static_cast<uint32_t>(max_bs), n,
                             reinterpret_cast<int32_t*>(d + off_x), dst, static_cast<uint32_t>(max_cand), d + off_ws,
                             ws_bytes, reinterpret_cast<uint32_t*>(dst + 1), st);
    if (rc != RPP_OK) throw fail(status_name(rc));
    int32_t res[2] = {0, 0};  // status, candidates found
    hip_check(hipMemcpyAsync(res, dst, 8, hipMemcpyDeviceToHost, st), "D2H flac status");
    ctx->sync();
    const uint64_t found = static_cast<uint32_t>(res[1]);
    if (found > max_cand) {
      if (attempt > 0 || too_wide(found)) throw fail(std::to_string(found) + " frame candidates");
      max_cand = found + 64;
      continue;
    }
    if (res[0] != RPP_OK) throw fail(status_name(res[0]));
    rc = rpp_pcm_pack(&pf, reinterpret_cast<int32_t const*>(d + off_x), d + off_pcm, nvals, st);
    if (rc != RPP_OK) throw fail(status_name(rc));
    hip_check(hipMemcpyAsync(target_->data(), d + off_pcm, frame_.uncompressed_bytes, hipMemcpyDeviceToHost, st),
              "D2H flac pcm");
    ctx->sync();
    return true;
  }
}

std::vector<uint8_t> flac_block_decompressor::decompress(std::span<uint8_t const> data) {
  flac_block_decompressor d{data};
  std::vector<uint8_t> out;
  d.start_decompression(&out);
  d.decompress_frame(d.uncompressed_size());
  return out;
}

}  // namespace ricepp_amd
