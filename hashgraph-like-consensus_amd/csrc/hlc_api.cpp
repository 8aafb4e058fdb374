// hlc_api.cpp -- the C ABI of include/hlc.h: context, device workspace, host<->device staging,
// and the orchestration of the kernels in hlc_prehash.hip / hlc_recover.hip.
#include <hip/hip_runtime.h>

#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hlc.h"
#include "hlc_kernels.h"

#if !defined(__HIP_DEVICE_COMPILE__) && defined(__x86_64__)
#include <immintrin.h>
#define HLC_HAVE_NT_COPY 1
#endif

namespace {

thread_local std::string g_err;

int set_err(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                                 \
  do {                                                                                               \
    hipError_t e_ = (expr);                                                                          \
    if (e_ != hipSuccess)                                                                            \
      return set_err(e_ == hipErrorOutOfMemory ? HLC_ENOMEM : HLC_EDEVICE,                           \
                     std::string(#expr) + ": " + hipGetErrorString(e_));                             \
  } while (0)

#define CHK(expr)            \
  do {                       \
    int rc_ = (expr);        \
    if (rc_ != 0) return rc_; \
  } while (0)

struct DBuf {
  void* p = nullptr;
  size_t cap = 0;
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
  int ensure(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) {
      (void)hipFree(p);
      p = nullptr;
      cap = 0;
    }
    size_t want = bytes + bytes / 4 + 256;
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {
      p = nullptr;
      return set_err(HLC_ENOMEM, std::string("hipMalloc failed: ") + hipGetErrorString(e));
    }
    cap = want;
    return 0;
  }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

// Page-locked host memory (the host-buffer entries' staging buffers: DMA runs asynchronously from it).
struct PBuf {
  void* p = nullptr;
  size_t cap = 0;
  ~PBuf() {
    if (p) (void)hipHostFree(p);
  }
  int ensure(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = bytes + bytes / 4 + 4096;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e != hipSuccess) {
      p = nullptr;
      return set_err(HLC_ENOMEM, std::string("hipHostMalloc failed: ") + hipGetErrorString(e));
    }
    cap = want;
    return 0;
  }
  uint8_t* at(size_t off) const { return static_cast<uint8_t*>(p) + off; }
};

// The host-buffer entries' staging copies into page-locked memory (HLC_NT_COPY, default 1): 32-byte
// non-temporal stores when the CPU has AVX2 -- the staging buffer is written once and next read by the
// DMA engine, so the copy need not read its destination lines into the cache first (a plain memcpy of
// the pool's 16-256 KB pieces stays below glibc's non-temporal threshold and does); sfence at the end,
// before the pool reports the piece done and the DMA of it is enqueued.
#ifdef HLC_HAVE_NT_COPY
__attribute__((target("avx2"))) void copy_nt_avx2(uint8_t* dst, const uint8_t* src, size_t n) {
  const size_t head = (32 - ((uintptr_t)dst & 31)) & 31;
  std::memcpy(dst, src, head);
  dst += head;
  src += head;
  n -= head;
  size_t i = 0;
  for (; i + 128 <= n; i += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 64));
    const __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 96), d);
  }
  std::memcpy(dst + i, src + i, n - i);
  _mm_sfence();
}
#endif
bool cpu_has_avx2() {
#ifdef HLC_HAVE_NT_COPY
  return __builtin_cpu_supports("avx2");
#else
  return false;
#endif
}
// nt: the context's HLC_OPT_NT_COPY (and the CPU has AVX2)
void stage_copy(uint8_t* dst, const uint8_t* src, size_t n, bool nt) {
#ifdef HLC_HAVE_NT_COPY
  if (nt && n >= 4096) {
    copy_nt_avx2(dst, src, n);
    return;
  }
#endif
  std::memcpy(dst, src, n);
}

// A small host worker pool for the host-buffer entries' field checks and staging copies: run(fn) calls
// fn(chunk, chunks()) once for every chunk, on the workers and the calling thread, and returns when all
// are done.  Threads take chunks (4 per thread) from a shared counter, so a thread the OS holds back
// (the box's CPU quota is shared with the caller's own threads) delays one chunk, not 1/threads of
// the job.
class HostPool {
 public:
  // cpus non-empty: every worker is bound to that CPU set (the GPU's NUMA node, host_pool_cpus)
  explicit HostPool(int workers, const std::vector<int>& cpus = {}) {
    for (int i = 0; i < workers; ++i)
      th_.emplace_back([this, cpus] {
        if (!cpus.empty()) {
          cpu_set_t set;
          CPU_ZERO(&set);
          for (int c : cpus) CPU_SET(c, &set);
          (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
        }
        loop();
      });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> l(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int threads() const { return (int)th_.size() + 1; }
  // moves every worker to another CPU set (empty: any CPU of the process's affinity mask)
  void rebind(const std::vector<int>& cpus) {
    cpu_set_t set;
    CPU_ZERO(&set);
    if (cpus.empty()) {
      if (sched_getaffinity(0, sizeof set, &set) != 0) return;
    } else {
      for (int c : cpus) CPU_SET(c, &set);
    }
    for (auto& t : th_) (void)pthread_setaffinity_np(t.native_handle(), sizeof set, &set);
  }
  int chunks() const { return 4 * threads(); }
  void run(const std::function<void(int, int)>& fn) {
    {
      std::lock_guard<std::mutex> l(m_);
      fn_ = &fn;
      next_.store(0, std::memory_order_relaxed);
      pending_ = (int)th_.size();
      ++gen_;
    }
    cv_.notify_all();
    work(fn);
    std::unique_lock<std::mutex> l(m_);
    done_.wait(l, [&] { return pending_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work(const std::function<void(int, int)>& fn) {
    const int C = chunks();
    for (int k = next_.fetch_add(1, std::memory_order_relaxed); k < C; k = next_.fetch_add(1, std::memory_order_relaxed))
      fn(k, C);
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int, int)>* f;
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        f = fn_;
      }
      work(*f);
      std::lock_guard<std::mutex> l(m_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::atomic<int> next_{0};
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int, int)>* fn_ = nullptr;
  int pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// A context's tunables (hlc_ctx_set_option, HLC_OPT_* in hlc.h).  Their defaults come from the
// environment, read once when the context is created (read_env, the only getenv site of the library) --
// never inside a call, so an embedder's threads may setenv freely and the Rust binding sets them per
// context.
struct Options {
  int host_threads = 16;      // HLC_OPT_HOST_THREADS: staging threads incl. the caller
  int pool_bind = HLC_POOL_BIND_NONE;  // HLC_OPT_POOL_BIND (unbound measured best)
  int nt_copy = 1;            // HLC_OPT_NT_COPY: non-temporal staging copies (AVX2)
  std::vector<uint64_t> split_votes{98304, 196608};  // HLC_OPT_SPLIT_VOTES (split_ranges)
  int host_trace = 0;         // HLC_OPT_HOST_TRACE
  int first_batch = 1;        // HLC_OPT_FIRST_BATCH
  int rest_pieces = 3;        // HLC_OPT_REST_PIECES
  std::vector<uint64_t> wire_split_bytes{8ull << 20, 16ull << 20, 24ull << 20, 32ull << 20};  // (wire_ranges)
  uint64_t wire_front_cap = 1536;  // HLC_OPT_WIRE_FRONT_CAP (waves; 0 = full grids)
  uint64_t wire_chunk = 4ull << 20;  // HLC_OPT_WIRE_CHUNK
  int rec_force_exact = 0;    // HLC_OPT_REC_FORCE_EXACT: every vote through the checked chains (tests)
  int serial_stages = 0;      // HLC_OPT_SERIAL_STAGES: prep + main after the prehash on one stream
  int wire_pipeline = 1;      // HLC_OPT_WIRE_PIPELINE: 0 = the unpipelined wire host entry (A/B arm)
  int wire_walk = -1;         // HLC_OPT_WIRE_WALK: -1 the build's default walker, 0 per lane, 1 LDS
  int early_comb = 1;         // HLC_OPT_EARLY_COMB bits: 1 device-resident calls (+0.65%), 2 host-buffer calls
};

// The CPUs the cgroup (v2) quota grants the process, or 0 when there is none.
double cgroup_cpu_quota() {
  std::FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r");
  if (!f) return 0;
  char q[64] = {0};
  double per = 0;
  const int got = std::fscanf(f, "%63s %lf", q, &per);
  std::fclose(f);
  if (got != 2 || per <= 0 || std::strcmp(q, "max") == 0) return 0;
  return std::atof(q) / per;
}

std::vector<uint64_t> parse_list(const char* p) {
  std::vector<uint64_t> out;
  while (*p) {
    char* end = nullptr;
    const uint64_t x = std::strtoull(p, &end, 10);
    if (end == p) break;
    out.push_back(x);
    p = *end == ',' ? end + 1 : end;
  }
  return out;
}

// The defaults of a new context's options, from the environment (the HLC_* variables the tools set).
// Staging workers (HLC_HOST_THREADS): by default 16 -- the GPU box's CPU share per GPU -- capped by the
// hardware threads and by this process's share of the CPUs: the cgroup quota (or the hardware threads)
// divided by the ranks on the node (LOCAL_WORLD_SIZE, set by torch.distributed.run), so that 8 ranks do
// not run 8 x 16 staging threads on one node's quota.  Measured on two boxes with the chunked pool: 16
// threads 86.9 / 88.3 M votes/s, 12: 86.0 / 88.0, 8: 85.2 / 87.1 (profiles/r04/host_pool_threads.txt).
Options read_env() {
  Options o;
  const char* e;
  const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
  int ranks = 1;
  if ((e = std::getenv("LOCAL_WORLD_SIZE"))) ranks = std::max(1, std::atoi(e));
  const double quota = cgroup_cpu_quota();
  const double share = (quota > 0 ? std::min(quota, (double)hw) : (double)hw) / ranks;
  o.host_threads = std::max(1, std::min({16, hw, (int)(share + 1e-9)}));
  if ((e = std::getenv("HLC_HOST_THREADS"))) o.host_threads = std::max(1, std::min(std::atoi(e), 64));
  if ((e = std::getenv("HLC_POOL_BIND"))) o.pool_bind = std::max(0, std::min(std::atoi(e), 2));
  if ((e = std::getenv("HLC_NT_COPY"))) o.nt_copy = std::atoi(e) != 0;
  if ((e = std::getenv("HLC_SPLIT_VOTES"))) o.split_votes = parse_list(e);
  if ((e = std::getenv("HLC_HOST_TRACE"))) o.host_trace = std::max(0, std::min(std::atoi(e), 2));
  if ((e = std::getenv("HLC_FIRST_BATCH"))) o.first_batch = std::max(0, std::atoi(e));
  if ((e = std::getenv("HLC_REST_PIECES"))) o.rest_pieces = std::max(1, std::min(std::atoi(e), 64));
  if ((e = std::getenv("HLC_WIRE_SPLIT_BYTES"))) o.wire_split_bytes = parse_list(e);
  if ((e = std::getenv("HLC_WIRE_FRONT_CAP"))) o.wire_front_cap = (uint64_t)std::max(0LL, std::atoll(e));
  if ((e = std::getenv("HLC_WIRE_CHUNK"))) o.wire_chunk = std::max<uint64_t>(std::strtoull(e, nullptr, 10), 4096);
  if ((e = std::getenv("HLC_REC_FORCE_EXACT"))) o.rec_force_exact = std::atoi(e) != 0;
  if ((e = std::getenv("HLC_SERIAL_STAGES"))) o.serial_stages = std::atoi(e) != 0;
  if ((e = std::getenv("HLC_WIRE_PIPELINE"))) o.wire_pipeline = std::atoi(e) != 0;
  if ((e = std::getenv("HLC_WIRE_WALK"))) o.wire_walk = std::strcmp(e, "lane") == 0 ? 0 : 1;
  if ((e = std::getenv("HLC_EARLY_COMB"))) o.early_comb = std::max(0, std::min(std::atoi(e), 3));
  return o;
}

// The fixed-base tables: the signing comb (32 x 256 affine points, 512 KiB) and the recovery's u1 G comb
// it is built from (hlc_recover.hpp: 11 windows x 2^23 affine points of 64 B = 5.9 GB at W = 24).  Both are
// read-only once built, so there is one pair per device per process, shared by every context on that
// device and freed with the last of them: a second context costs no table memory and no build.
struct GenTables {
  int device = -1;
  void* fb = nullptr;
  void* g = nullptr;
  ~GenTables() {
    if (!fb && !g) return;
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    if (fb) (void)hipFree(fb);
    if (g) (void)hipFree(g);
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);  // the caller's current device, unchanged
  }
};
std::mutex g_gen_mu;
std::map<int, std::weak_ptr<GenTables>>* g_gen = new std::map<int, std::weak_ptr<GenTables>>();  // (never freed:
                                                   // contexts destroyed by static destructors still find it)

// The device's tables (built on `s` and synchronised on first use; the caller has set `device`).
int gen_tables(int device, hipStream_t s, std::shared_ptr<GenTables>& out) {
  std::lock_guard<std::mutex> lk(g_gen_mu);
  if ((out = (*g_gen)[device].lock())) return 0;
  auto t = std::make_shared<GenTables>();
  t->device = device;
  const size_t gbytes = hlc::gcomb_words() * sizeof(uint32_t);
  hipError_t e = hipMalloc(&t->fb, hlc::FBTAB_WORDS * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&t->g, gbytes);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_err(HLC_ENOMEM, "fixed-base table allocation (" + std::to_string(gbytes >> 20) +
                                   " MiB u1 G comb) failed: " + hipGetErrorString(e));
  }
  hlc::launch_build_fbtab(reinterpret_cast<uint32_t*>(t->fb), s);
  hlc::launch_build_gcomb(reinterpret_cast<uint32_t*>(t->g), reinterpret_cast<const uint32_t*>(t->fb), s);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return set_err(HLC_EDEVICE, "generator table construction failed");
  (*g_gen)[device] = t;
  out = std::move(t);
  return 0;
}

}  // namespace

struct hlc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t aux = nullptr;                        // the recovery prep stage, concurrent with the prehash
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;  // caller stream -> aux -> caller stream
  hipEvent_t ev_prep = nullptr;  // aux: the recovery's prep stage done (HLC_OPT_EARLY_COMB)
  std::mutex mu;
  std::shared_ptr<GenTables> gen;  // the device's fixed-base tables (gen_tables), shared with its other contexts
  const uint32_t* gtab = nullptr;  // the u1 G comb (gen->g)
  const uint32_t* fbtab = nullptr; // the signing comb (gen->fb)
  DBuf rec_scratch, rec_work;
  uint64_t rec_lanes = 0;
  Options opt;  // hlc_ctx_set_option; defaults from the environment at creation (read_env)
  // hlc_validate_proposals (host buffers): a second recovery slot (stream, per-lane scratch, per-vote
  // records) so that two k_rec_main grids over the two vote ranges of a call overlap; an upload stream;
  // the page-locked staging of the inputs and outputs and their device copies (allocated on first use)
  hipStream_t aux2 = nullptr, copy = nullptr;
  hipStream_t dec = nullptr, wlk = nullptr;  // wire host entry: the ranges' decode and walks (greatest priority)
  DBuf rec_scratch2;
  std::vector<std::unique_ptr<DBuf>> rec_works;  // each recovery range's work list, prefix products, counters
  PBuf pin_in, pin_out;
  DBuf dev_in, dev_out;
  std::vector<hipEvent_t> ev_up, ev_main;  // per recovery range: inputs landed, main stage done
  std::vector<hipEvent_t> ev_prepk;        // per recovery range: prep stage done (early comb, host entries)
  std::vector<hipEvent_t> ev_cnt, ev_dec;  // wire host entry, per message range: vote count read back, decoded
  PBuf pin_cnt;                            // wire host entry: the ranges' vote counts (page-locked)
  uint64_t wire_hint = 0;                  // wire host entry: the largest vote count a call decoded
  std::string last_trace;                  // the last host-buffer call's host trace JSON (HLC_OPT_HOST_TRACE)
  hipEvent_t ev_rest = nullptr, ev_done = nullptr;
  std::unique_ptr<HostPool> pool;  // staging workers (HLC_HOST_THREADS)
  std::vector<int> pool_cpus;      // the CPU set its workers are bound to now (empty: unbound)
  int pool_node = -2;              // the NUMA node they are bound to (-1: unbound, -2: not yet decided)
  // staged host inputs (host-buffer entry points)
  DBuf in_vote_id, in_pid, in_ts, in_vote, in_bytes, in_off, in_len, in_props;
  DBuf in_off2, in_len2, in_off3, in_len3, in_priv, byz_key, in_verdict;
  // outputs staged on device
  DBuf out_res, out_status, out_reason, out_rec, out_misc;
  // internal workspace
  // measurement hooks
  int timing = 0;  // 0, HLC_TIMING_ALL or HLC_TIMING_RECOVERY (hlc_ctx_set_kernel_timing)
  bool timing_all() const { return timing == HLC_TIMING_ALL; }
  bool clock_probe = false;  // hlc_ctx_set_clock_probe: k_rec_main's per-wave clock stamps into clk_buf
  DBuf clk_buf;
  uint64_t clk_waves = 0;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> rec_ev, rec_prep_ev, call_ev, chain_ev, chain_aux_ev;
  hipEvent_t take_event() {
    if (ev_pool.empty()) {
      hipEvent_t e = nullptr;
      (void)hipEventCreate(&e);
      return e;
    }
    hipEvent_t e = ev_pool.back();
    ev_pool.pop_back();
    return e;
  }
  ~hlc_ctx() {
    for (auto e : ev_pool) (void)hipEventDestroy(e);
    for (auto& pr : rec_ev) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    for (auto& pr : rec_prep_ev) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    for (auto& pr : chain_aux_ev) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    for (hipEvent_t e : ev_up) (void)hipEventDestroy(e);
    for (hipEvent_t e : ev_main) (void)hipEventDestroy(e);
    for (hipEvent_t e : ev_prepk) (void)hipEventDestroy(e);
    for (hipEvent_t e : ev_cnt) (void)hipEventDestroy(e);
    for (hipEvent_t e : ev_dec) (void)hipEventDestroy(e);
    for (hipEvent_t e : {ev_rest, ev_done})
      if (e) (void)hipEventDestroy(e);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
    if (ev_prep) (void)hipEventDestroy(ev_prep);
    for (auto& pr : call_ev) (void)hipEventDestroy(pr.first);  // (pr.second is chain_ev's)
    for (auto& pr : chain_ev) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
  }
  DBuf vote_prop, sha_sz, sha_off, kec_sz, kec_off, sha_buf, kec_buf, sha_dig, kec_dig, pre, pre_reason,
      verify, status, reason, chain_code, chain_tab, dup_tab, red, scan_tmp, totals, flag;
  // wire decode: staged inputs, walk / record workspace, decoded votes (hlc_votes SoA over the wire bytes)
  DBuf w_wire, w_moff, w_mlen, w_scope, w_vcount, w_vbegin, w_vrec_off, w_vrec_len, w_vrec_msg, w_first_bad,
      w_vote_err, w_props, w_wout, w_res, w_slab_off, w_slab_len, w_big;
  DBuf w_huge, h_next, h_jump, h_mark, h_st, h_flag, h_rank, h_scan, h_off, h_len, h_save;
  DBuf w_vid, w_pid, w_ts, w_vote, w_foff, w_flen;
  // streaming votes
  DBuf s_vsess, s_sessions, s_owners, s_osess, s_props, s_keys, s_iota, s_order, s_segb, s_sege, s_tab, s_sort_tmp,
      s_st, s_tr, s_ins, s_slot, s_dup;
};

namespace {

// the context's second stream (the recovery's prep / main stages)
hipError_t create_aux(hlc_ctx* c) { return hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking); }

int activate(hlc_ctx* ctx) {
  HIPCHK(hipSetDevice(ctx->device));
  return 0;
}

template <class T>
int upload(DBuf& b, const T* host, size_t count, hipStream_t s) {
  CHK(b.ensure(count * sizeof(T) + 16));
  if (count) HIPCHK(hipMemcpyAsync(b.p, host, count * sizeof(T), hipMemcpyHostToDevice, s));
  return 0;
}

// Prefix sums of message sizes + device->host read of the totals (one sync).
int scan_sizes(hlc_ctx* c, uint64_t n, const uint64_t* sz, uint64_t* off, uint64_t* total, hipStream_t s) {
  size_t tb = 0;
  HIPCHK(hlc::launch_exclusive_scan(sz, off, n, nullptr, tb, s));
  CHK(c->scan_tmp.ensure(tb + 16));
  HIPCHK(hlc::launch_exclusive_scan(sz, off, n, c->scan_tmp.p, tb, s));
  HIPCHK(hipGetLastError());
  CHK(c->totals.ensure(4 * sizeof(uint64_t)));
  uint64_t* t = c->totals.as<uint64_t>();
  HIPCHK(hipMemcpyAsync(t, off + (n - 1), sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
  HIPCHK(hipMemcpyAsync(t + 1, sz + (n - 1), sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
  uint64_t h[2];
  HIPCHK(hipMemcpyAsync(h, t, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  *total = h[0] + h[1];
  return 0;
}

// Builds + hashes the vote messages: sha_dig (vote hash) and kec_dig (EIP-191 prehash).
int run_prehash(hlc_ctx* c, const hlc_votes* dv, uint64_t n, int mode, const uint8_t* bytes,
                const uint64_t* pay_off, const uint32_t* pay_len, hipStream_t s) {
  CHK(c->sha_sz.ensure(n * 8));
  CHK(c->sha_off.ensure(n * 8));
  CHK(c->kec_sz.ensure(n * 8));
  CHK(c->kec_off.ensure(n * 8));
  hlc::launch_msg_sizes(dv, n, pay_off, pay_len, mode, c->sha_sz.as<uint64_t>(), c->kec_sz.as<uint64_t>(), s);
  uint64_t sha_total = 0, kec_total = 0;
  if (mode == hlc::MSG_VOTE) CHK(scan_sizes(c, n, c->sha_sz.as<uint64_t>(), c->sha_off.as<uint64_t>(), &sha_total, s));
  CHK(scan_sizes(c, n, c->kec_sz.as<uint64_t>(), c->kec_off.as<uint64_t>(), &kec_total, s));
  CHK(c->sha_buf.ensure(sha_total + 64));
  CHK(c->kec_buf.ensure(kec_total + 136));
  CHK(c->sha_dig.ensure(n * 32));
  CHK(c->kec_dig.ensure(n * 32));
  hlc::launch_build_msgs(dv, n, bytes, pay_off, pay_len, mode, c->sha_off.as<uint64_t>(), c->sha_sz.as<uint64_t>(),
                         c->sha_buf.as<uint8_t>(), c->kec_off.as<uint64_t>(), c->kec_sz.as<uint64_t>(),
                         c->kec_buf.as<uint8_t>(), s);
  if (mode == hlc::MSG_VOTE)
    hlc::launch_sha_blocks(n, c->sha_off.as<uint64_t>(), c->sha_sz.as<uint64_t>(), c->sha_buf.as<uint8_t>(),
                           c->sha_dig.as<uint32_t>(), s);
  hlc::launch_keccak_blocks(n, c->kec_off.as<uint64_t>(), c->kec_sz.as<uint64_t>(), c->kec_buf.as<uint8_t>(),
                            c->kec_dig.as<uint32_t>(), s);
  HIPCHK(hipGetLastError());
  return 0;
}

int ensure_recover_scratch(hlc_ctx* c) {
  if (c->rec_lanes) return 0;
  uint64_t lanes = hlc::recover_grid_lanes();
  CHK(c->rec_scratch.ensure(lanes * hlc::recover_scratch_words() * sizeof(uint32_t)));
  c->rec_lanes = lanes;
  return 0;
}

int ensure_fbtab(hlc_ctx* c) {
  return c->fbtab ? 0 : set_err(HLC_EINVAL, "context without its fixed-base tables");  // (built at creation)
}

// A recovery range whose front half (k_rec_prep + k_rec_main over votes [v0, v1), records in the
// call's rec_work) the caller has already enqueued on a stream of its own; `done` fires when that
// main stage ends.
struct RecFront {
  uint64_t v0, v1;
  hipEvent_t done;
  hipEvent_t prep;  // the range's k_rec_prep done
};

// Per-vote validate_vote stage (utils.rs:127-171; plus the proposal_id match of utils.rs:113-115)
// for votes already mapped to proposals (vote_prop, NO_PROP = skip): fused LDS prehash, the
// streaming general path for oversize votes (skipped on the device when no vote needs it),
// signature recovery, status assembly.  c->flag must hold the flags of the mapping step (cleared
// or set by launch_assign_props).  Everything is enqueued on `s` (and the context's aux stream,
// forked from and joined back into `s`): no host synchronisation.
// chain_code != nullptr: also the small proposals' chain / duplicate / YES kernel (it needs no
// vote statuses), on `s` beside the recovery's main stage.
// fronts != nullptr (hlc_validate_proposals over host buffers): the recovery's front halves are
// already in flight over those ranges (validate_host); one finish over all votes waits for them.
// (One finish, not one per range: its k_rec_final / k_rec_addr are short low-occupancy kernels, and
// per range they cost 0.95 ms against 0.67 ms for one launch over 640k votes.)
// verdicts != nullptr (the *_verdicts entries, any ConsensusSignatureScheme): the scheme step is the
// caller's per-vote verdict; the prehash runs without the Ethereum checks and keccak, and no recovery runs.
// aux_tables != nullptr: the large-proposal chain / duplicate tables' launcher (validate_device); with
// the early comb it is enqueued on the aux stream behind k_rec_main, where it runs beside the comb
// instead of on the launch stream's critical path, and *tables_done is set.
// fork_recorded: validate_device bound c->ev_fork to its last kernel on `s` (no marker needed here) and
// cleared the prep stage's work counters (hlc::recover_counters) in k_red_init.
using TablesLaunch = std::function<void(hipStream_t, const hlc::KEv*)>;
int vote_stage(hlc_ctx* c, const hlc_votes* dv, const uint32_t* vote_prop, const hlc_proposal* dprops, uint64_t np,
               uint64_t now, uint8_t* status, uint8_t* reason, uint8_t* drec, uint32_t* red, uint8_t* chain_code,
               hipStream_t s, const RecFront* fronts = nullptr, int nfronts = 0, uint64_t rec_stride = 0,
               const uint8_t* verdicts = nullptr, const TablesLaunch* aux_tables = nullptr,
               bool* tables_done = nullptr, bool fork_recorded = false) {
  const uint64_t n = dv->n;
  CHK(c->pre.ensure(n));
  CHK(c->pre_reason.ensure(n));
  if (verdicts) {
    hlc::launch_prehash_fused(dv, n, vote_prop, dprops, nullptr, c->pre.as<uint8_t>(), c->pre_reason.as<uint8_t>(),
                              c->flag.as<uint32_t>(), s, false);
    hlc::launch_prehash_stream(dv, n, vote_prop, dprops, c->flag.as<uint32_t>(), nullptr, c->pre.as<uint8_t>(),
                               c->pre_reason.as<uint8_t>(), s, false);
    if (chain_code) hlc::launch_chain_small(dv, dprops, np, chain_code, red, s);
    hlc::launch_vote_status(dv, n, vote_prop, dprops, now, c->pre.as<uint8_t>(), c->pre_reason.as<uint8_t>(), verdicts,
                            status, reason, red, s);
    HIPCHK(hipGetLastError());
    return 0;
  }
  CHK(c->verify.ensure(n));
  CHK(c->kec_dig.ensure(n * 32));
  CHK(ensure_recover_scratch(c));
  // the vote statuses are written by the finish's last kernel (k_rec_addr), not by a k_vote_status after it
  const hlc::VoteStatusArgs sa{*dv, vote_prop, dprops, now, c->pre_reason.as<uint8_t>(), status, reason, red};
  // (fronts: the ranges' records are in flight in rec_work, sized by the caller)
  if (!fronts) CHK(c->rec_work.ensure(hlc::recover_work_words(n) * sizeof(uint32_t)));
  // The recovery's prep stage (signature parse, batched r^-1, GLV digits) and main stage (R, its
  // table, the u2 R chain: ~93% of the recovery) need only the signatures, so they run on the
  // context's aux stream while the prehash kernels (and the small-proposal chain kernel) run on
  // `s`; `s` waits for them before the finish (u1 G with u1 = -z/r from the prehash, Z^-1,
  // address).  Measured recovery time = prep bracket (aux) + main start (aux) .. finish end (s).
  // (HLC_SERIAL_STAGES=1: everything on `s`, prep + main after the prehash and the chain kernel --
  // the measurement of k_rec_main running alone)
  hipStream_t aux = c->opt.serial_stages ? s : c->aux;
  // the recovery bracket: k_rec_prep's start .. k_rec_addr's end, both bound to the dispatches
  hipEvent_t p0 = nullptr, r1 = nullptr;
  if (c->timing && !fronts) {
    p0 = c->take_event();
    r1 = c->take_event();
  }
  // HLC_OPT_EARLY_COMB: u1 G (k_rec_ucomb) is enqueued on `s` behind the prehash and the prep stage;
  // k_rec_main's persistent grid holds every register until its tail, so the comb's waves take the
  // slots its waves leave, instead of starting after its last one
  const bool early = !fronts && (c->opt.early_comb & 1) && !c->opt.serial_stages;
  // the prep stage's completion (early comb: what `s` waits on), bound to k_rec_prep's dispatch
  const hipEvent_t prep_done = early ? c->ev_prep : nullptr;
  auto launch_ucomb = [&]() -> int {
    HIPCHK(hipStreamWaitEvent(s, prep_done, 0));
    hlc::launch_recover_ucomb(n, c->pre.as<uint8_t>(), c->kec_dig.as<uint32_t>(), c->gtab,
                              c->rec_work.as<uint32_t>(), s, c->opt.rec_force_exact);
    return 0;
  };
  auto prehash_and_chain = [&]() -> int {
    hlc::launch_prehash_fused(dv, n, vote_prop, dprops, c->kec_dig.as<uint32_t>(), c->pre.as<uint8_t>(),
                              c->pre_reason.as<uint8_t>(), c->flag.as<uint32_t>(), s);
    hlc::launch_prehash_stream(dv, n, vote_prop, dprops, c->flag.as<uint32_t>(), c->kec_dig.as<uint32_t>(),
                               c->pre.as<uint8_t>(), c->pre_reason.as<uint8_t>(), s);
    if (drec) HIPCHK(hipMemsetAsync(drec, 0, n * 20, s));
    if (chain_code) {
      hlc::KEv cs;
      if (c->timing_all()) {
        cs = hlc::KEv{c->take_event(), c->take_event()};
        c->chain_aux_ev.emplace_back(cs.start, cs.stop);
      }
      hlc::launch_chain_small(dv, dprops, np, chain_code, red, s, &cs);
    }
    return 0;
  };
  if (fronts) {
    CHK(prehash_and_chain());
    // HLC_OPT_EARLY_COMB bit 1: u1 G behind the prehash and every range's prep stage, in the last
    // range's k_rec_main tail
    const bool early_host = (c->opt.early_comb & 2) != 0;
    if (early_host) {
      for (int k = 0; k < nfronts; ++k) HIPCHK(hipStreamWaitEvent(s, fronts[k].prep, 0));
      hlc::launch_recover_ucomb(n, c->pre.as<uint8_t>(), c->kec_dig.as<uint32_t>(), c->gtab,
                                c->rec_work.as<uint32_t>(), s, c->opt.rec_force_exact, rec_stride);
    }
    for (int k = 0; k < nfronts; ++k) HIPCHK(hipStreamWaitEvent(s, fronts[k].done, 0));
    hlc::launch_recover_finish(n, c->pre.as<uint8_t>(), c->kec_dig.as<uint32_t>(), dv->bytes,
                               dv->field_off + HLC_F_OWNER, HLC_NFIELDS, c->gtab,
                               c->rec_work.as<uint32_t>(), c->verify.as<uint8_t>(), drec, s, c->opt.rec_force_exact,
                               rec_stride, early_host, nullptr, &sa);
    HIPCHK(hipGetLastError());
    return 0;
  }
  if (c->opt.serial_stages) {
    CHK(prehash_and_chain());
  } else {
    if (!fork_recorded) HIPCHK(hipEventRecord(c->ev_fork, s));
    HIPCHK(hipStreamWaitEvent(aux, c->ev_fork, 0));
  }
  // votes the checks before the signature reject (proposal_id mismatch, empty owner / vote_hash,
  // no covering proposal) are not recovered: vote_prop exists before the fork
  const hlc::RecSkip skip{vote_prop, dprops, dv->proposal_id, dv->field_len};
  const hlc::KEv pk{p0, prep_done};
  hlc::launch_recover_prep(n, dv->bytes, dv->field_off + HLC_F_SIGNATURE, HLC_NFIELDS, dv->field_len + HLC_F_SIGNATURE,
                           HLC_NFIELDS, c->rec_work.as<uint32_t>(), aux, &skip, nullptr, &pk, fork_recorded);
  unsigned long long* clk = nullptr;
  if (c->clock_probe) {
    CHK(c->clk_buf.ensure((c->rec_lanes / 64) * 32 + 32));
    HIPCHK(hipMemsetAsync(c->clk_buf.p, 0, (c->rec_lanes / 64) * 32, aux));
    clk = c->clk_buf.as<unsigned long long>();
  }
  // the join `s` waits on before the finish: k_rec_main's completion, or (early comb) that of the
  // large-proposal tables enqueued behind it on aux -- a timing event when their bracket is timed
  const bool tables_aux = early && aux_tables;
  hipEvent_t t0 = nullptr, join = c->opt.serial_stages ? nullptr : c->ev_join;
  if (tables_aux && c->timing_all()) {
    t0 = c->take_event();
    join = c->take_event();
    c->chain_aux_ev.emplace_back(t0, join);
  }
  const hlc::KEv mk{nullptr, tables_aux ? nullptr : join};
  hlc::launch_recover_main(n, dv->bytes, dv->field_off + HLC_F_SIGNATURE, HLC_NFIELDS, c->rec_scratch.as<uint32_t>(),
                           c->rec_lanes, c->rec_work.as<uint32_t>(), aux, c->opt.rec_force_exact, nullptr, clk,
                           clk ? &c->clk_waves : nullptr, &mk);
  if (tables_aux) {
    const hlc::KEv tk{t0, join};
    (*aux_tables)(aux, &tk);
    if (tables_done) *tables_done = true;
  }
  if (!c->opt.serial_stages) {
    CHK(prehash_and_chain());
    if (early) CHK(launch_ucomb());  // after the small-proposal chain kernel (before it: -0.4 to -1.1%)
    HIPCHK(hipStreamWaitEvent(s, join, 0));
  }
  const hlc::KEv fk{nullptr, r1};
  hlc::launch_recover_finish(n, c->pre.as<uint8_t>(), c->kec_dig.as<uint32_t>(), dv->bytes, dv->field_off + HLC_F_OWNER,
                             HLC_NFIELDS, c->gtab, c->rec_work.as<uint32_t>(), c->verify.as<uint8_t>(),
                             drec, s, c->opt.rec_force_exact, 0, early, &fk, &sa);
  if (c->timing) c->rec_ev.emplace_back(p0, r1);
  HIPCHK(hipGetLastError());
  return 0;
}

// The device workspace validate_device() needs for up to n votes and np proposals (grown on demand
// otherwise): hlc_ctx_reserve, and the pipeline's children before their first chunk, so that no
// buffer is reallocated while a chunk is in flight.
int reserve_validate(hlc_ctx* c, uint64_t n, uint64_t np) {
  CHK(ensure_recover_scratch(c));
  CHK(c->rec_work.ensure(hlc::recover_work_words(n) * sizeof(uint32_t)));
  CHK(c->kec_dig.ensure(n * 32));
  for (DBuf* b : {&c->pre, &c->pre_reason, &c->verify, &c->status, &c->reason, &c->chain_code}) CHK(b->ensure(n + 1));
  CHK(c->vote_prop.ensure(n * 4 + 4));
  uint64_t cap = 64;
  while (cap < 2 * n) cap <<= 1;
  CHK(c->chain_tab.ensure(cap * 4));
  CHK(c->dup_tab.ensure(cap * 4));
  CHK(c->red.ensure(np * 16 + 16));
  CHK(c->flag.ensure(16));
  return 0;
}

// Device-resident validate-many (every pointer is device memory).
int validate_device(hlc_ctx* c, const hlc_votes* dv, const hlc_proposal* dprops, uint64_t np, uint64_t now,
                    hlc_result* dres, uint8_t* dstatus, uint8_t* dreason, uint8_t* drec, hipStream_t s,
                    const RecFront* fronts = nullptr, int nfronts = 0, uint64_t rec_stride = 0,
                    const uint8_t* verdicts = nullptr) {
  const uint64_t n = dv->n;
  if (n > 0xFFFFFFF0ull) return set_err(HLC_EINVAL, "too many votes in one call (max 2^32-16)");
  // timing: call0 .. ch1 (the call), ch0 .. ch1 (chain check + duplicates + tally), all bound to
  // kernel dispatches (hlc::KEv); ch1 is shared by the two brackets and owned by chain_ev
  hipEvent_t call0 = nullptr, ch0 = nullptr, ch1 = nullptr;
  if (c->timing_all()) {
    call0 = c->take_event();
    ch0 = c->take_event();
    ch1 = c->take_event();
  }
  CHK(c->vote_prop.ensure(n * 4 + 4));
  CHK(c->flag.ensure(16));
  CHK(c->red.ensure(np * 16 + 16));
  // per-proposal reduction records and the call's flag word in one launch, then the vote -> proposal map
  // the default recovery path (prepped): the aux stream's fork point bound to k_assign_props's dispatch,
  // and the prep stage's two work counters cleared here with the rest
  const bool bind_fork = n && !fronts && !verdicts && !c->opt.serial_stages;
  unsigned long long* rec_ctr = nullptr;
  if (bind_fork) {
    CHK(c->rec_work.ensure(hlc::recover_work_words(n) * sizeof(uint32_t)));
    rec_ctr = hlc::recover_counters(n, c->rec_work.as<uint32_t>());
  }
  const hlc::KEv rk{call0, nullptr};
  hlc::launch_red_init(c->red.as<uint32_t>(), np, s, c->flag.as<uint32_t>(), &rk, c->vote_prop.as<uint32_t>(), n,
                       rec_ctr);
  const hlc::KEv ak{nullptr, bind_fork ? c->ev_fork : nullptr};
  HIPCHK(hlc::launch_assign_props(dprops, np, dv->field_len, c->vote_prop.as<uint32_t>(), n, c->flag.as<uint32_t>(), s,
                                  &ak, true));
  uint8_t* status = dstatus;
  uint8_t* reason = dreason;
  if (!status) {
    CHK(c->status.ensure(n + 1));
    status = c->status.as<uint8_t>();
  }
  if (!reason) {
    CHK(c->reason.ensure(n + 1));
    reason = c->reason.as<uint8_t>();
  }
  CHK(c->chain_code.ensure(n + 1));
  // proposals > 512 votes use global chain / duplicate tables; the kernels are always enqueued and
  // do nothing unless k_assign_props raised FLAG_LARGE_PROPOSAL (no host read-back)
  uint64_t cap = 64;
  while (cap < 2 * n) cap <<= 1;
  CHK(c->chain_tab.ensure(cap * 4));
  CHK(c->dup_tab.ensure(cap * 4));
  const TablesLaunch tables = [&](hipStream_t st, const hlc::KEv* ev) {
    hlc::launch_tables(dv, n, c->vote_prop.as<uint32_t>(), dprops, c->chain_tab.as<uint32_t>(),
                       c->dup_tab.as<uint32_t>(), (uint32_t)(cap - 1), c->red.as<uint32_t>(), np, c->flag.as<uint32_t>(),
                       st, ev);
  };
  // the large proposals' chain check reads no vote status, only the tables: it follows them
  auto chain_check = [&](hipStream_t st, const hlc::KEv* ev) {
    hlc::launch_chain_check(dv, n, c->vote_prop.as<uint32_t>(), dprops, status, c->chain_tab.as<uint32_t>(),
                            c->dup_tab.as<uint32_t>(), (uint32_t)(cap - 1), c->chain_code.as<uint8_t>(),
                            c->red.as<uint32_t>(), np, c->flag.as<uint32_t>(), st, ev);
  };
  // early comb: the tables and the chain check behind k_rec_main on the aux stream (vote_stage), beside
  // the comb, so that only k_finalize follows the recovery's finish on `s`
  const TablesLaunch tables_check = [&](hipStream_t st, const hlc::KEv* ev) {
    const hlc::KEv first = hlc::kev_start(ev), last = hlc::kev_stop(ev);
    tables(st, &first);
    chain_check(st, &last);
  };
  bool tables_done = false;
  // (the small proposals' chain / duplicate / YES kernel runs inside vote_stage, beside the
  // recovery's main stage: the finish reports each proposal's first failing vote)
  if (n)
    CHK(vote_stage(c, dv, c->vote_prop.as<uint32_t>(), dprops, np, now, status, reason, drec, c->red.as<uint32_t>(),
                   c->chain_code.as<uint8_t>(), s, fronts, nfronts, rec_stride, verdicts, &tables_check,
                   &tables_done, bind_fork));
  // chain check + duplicate detection + tally (+ k_chain_small's and the aux tables' brackets in vote_stage)
  const hlc::KEv c0{ch0, nullptr}, c1{nullptr, ch1}, cf{ch0, ch1};
  if (!tables_done) {
    tables(s, &c0);
    chain_check(s, nullptr);
  }
  hlc::launch_finalize(dprops, np, now, status, reason, c->chain_code.as<uint8_t>(), c->red.as<uint32_t>(), dres, s,
                       tables_done ? &cf : &c1);
  HIPCHK(hipGetLastError());
  if (c->timing_all()) {
    c->chain_ev.emplace_back(ch0, ch1);
    c->call_ev.emplace_back(call0, ch1);
  }
  return 0;
}

// Device decode of n_msgs Proposal messages (all pointers device memory).  Fills the context's
// decoded-vote SoA (*dv, viewing `wire` as its byte arena), dprops / dwout (caller-provided
// device arrays of n_msgs), and *n_votes.  One host synchronisation (the vote total).
int decode_device(hlc_ctx* c, const uint8_t* wire, uint64_t wire_len, const uint64_t* moff, const uint32_t* mlen,
                  uint64_t nm, const hlc_scope_config* scope, uint64_t n_scope, hlc_proposal* dprops,
                  hlc_wire_proposal* dwout, hlc_votes* dv, uint64_t* n_votes, hipStream_t s) {
  CHK(c->w_vcount.ensure(nm * 8 + 8));
  CHK(c->w_vbegin.ensure(nm * 8 + 8));
  const uint64_t slab = hlc::wire_slab();
  CHK(c->w_slab_off.ensure(nm * slab * 8 + 8));
  CHK(c->w_slab_len.ensure(nm * slab * 4 + 4));
  CHK(c->w_big.ensure(16));
  uint64_t* vcount = c->w_vcount.as<uint64_t>();
  uint64_t* vbegin = c->w_vbegin.as<uint64_t>();
  CHK(c->w_huge.ensure(nm * 16 + 16));
  uint64_t nv = 0;
  uint32_t big = 0;
  // (message index, length) of the messages longer than wire_huge_threshold(): decoded by the
  // parallel boundary-discovery path instead of the walker.
  std::vector<uint64_t> huge;
  uint64_t huge_recs = 0;
  if (nm) {
    HIPCHK(hipMemsetAsync(c->w_big.p, 0, 4, s));
    HIPCHK(hipMemsetAsync(c->w_huge.p, 0, 8, s));
    hlc::launch_wire_touch(wire, wire_len, c->w_big.as<uint32_t>() + 1, s);
    hlc::launch_wire_walk(0, wire, moff, mlen, nm, vcount, nullptr, dwout, dprops, scope, n_scope,
                          c->w_slab_off.as<uint64_t>(), c->w_slab_len.as<uint32_t>(), c->w_big.as<uint32_t>(), nullptr,
                          nullptr, nullptr, c->w_huge.as<uint64_t>(), s, nullptr, c->opt.wire_walk);
    // The huge-message count rides on the vote-total synchronisation; only when a message took the
    // parallel path (skipped by the walker, vote_count 0 so far) is there a second round trip.
    auto scan_totals = [&](uint64_t* h) -> int {
      size_t tb = 0;
      HIPCHK(hlc::launch_exclusive_scan(vcount, vbegin, nm, nullptr, tb, s));
      CHK(c->scan_tmp.ensure(tb + 16));
      HIPCHK(hlc::launch_exclusive_scan(vcount, vbegin, nm, c->scan_tmp.p, tb, s));
      HIPCHK(hipMemcpyAsync(h, vbegin + (nm - 1), 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(h + 1, vcount + (nm - 1), 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(h + 2, c->w_big.p, 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(h + 3, c->w_huge.p, 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      return 0;
    };
    uint64_t h[4] = {0, 0, 0, 0};  // last begin, last count, big flag, huge count
    CHK(scan_totals(h));
    const uint64_t nh = h[3];
    if (nh) {
      huge.resize(2 * nh);
      HIPCHK(hipMemcpyAsync(huge.data(), c->w_huge.as<uint64_t>() + 1, 16 * nh, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      uint64_t maxlen = 0;
      for (uint64_t i = 0; i < nh; ++i) {
        maxlen = std::max(maxlen, huge[2 * i + 1]);
        huge_recs += huge[2 * i + 1] / 2 + 1;  // a field takes >= 2 bytes
      }
      const size_t tb = hlc::huge_scan_bytes((uint32_t)maxlen);
      CHK(c->h_next.ensure(maxlen * 4 + 16));
      CHK(c->h_jump.ensure(maxlen * 4 + 16));
      CHK(c->h_save.ensure(maxlen * 4 + 16));
      CHK(c->h_mark.ensure(maxlen + 16));
      CHK(c->h_st.ensure(64));
      CHK(c->h_flag.ensure(maxlen * 4 + 16));
      CHK(c->h_rank.ensure(maxlen * 4 + 16));
      CHK(c->h_scan.ensure(tb + 16));
      CHK(c->h_off.ensure(huge_recs * 8 + 8));
      CHK(c->h_len.ensure(huge_recs * 4 + 4));
      std::vector<uint64_t> moff_h(nh);
      for (uint64_t i = 0; i < nh; ++i)
        HIPCHK(hipMemcpyAsync(&moff_h[i], moff + huge[2 * i], 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      uint64_t hb = 0;
      for (uint64_t i = 0; i < nh; ++i) {
        const uint32_t len = (uint32_t)huge[2 * i + 1];
        if (hlc::launch_huge_decode(wire, huge[2 * i], moff_h[i], len, c->h_next.as<uint32_t>(),
                                    c->h_jump.as<uint32_t>(), c->h_save.as<uint32_t>(), c->h_mark.as<uint8_t>(),
                                    c->h_st.as<uint32_t>(), c->h_flag.as<uint32_t>(), c->h_rank.as<uint32_t>(),
                                    c->h_scan.p, tb, c->h_off.as<uint64_t>() + hb, c->h_len.as<uint32_t>() + hb, vcount,
                                    dwout, dprops, scope, n_scope, s) != 0)
          return set_err(HLC_EDEVICE, std::string("huge-message decode: ") + hipGetErrorString(hipGetLastError()));
        hb += len / 2 + 1;
      }
      h[0] = h[1] = h[2] = h[3] = 0;
      CHK(scan_totals(h));
    }
    nv = h[0] + h[1];
    big = (uint32_t)h[2];
  }
  if (nv > 0xFFFFFFF0ull) return set_err(HLC_EINVAL, "too many votes in one call (max 2^32-16)");
  CHK(c->w_vrec_off.ensure(nv * 8 + 8));
  CHK(c->w_vrec_len.ensure(nv * 4 + 4));
  CHK(c->w_vrec_msg.ensure(nv * 4 + 4));
  CHK(c->w_first_bad.ensure(nm * 4 + 4));
  CHK(c->w_vote_err.ensure(nv + 1));
  CHK(c->w_vid.ensure(nv * 4 + 4));
  CHK(c->w_pid.ensure(nv * 4 + 4));
  CHK(c->w_ts.ensure(nv * 8 + 8));
  CHK(c->w_vote.ensure(nv + 1));
  CHK(c->w_foff.ensure(nv * 8 * HLC_NFIELDS + 8));
  CHK(c->w_flen.ensure(nv * 4 * HLC_NFIELDS + 4));
  dv->n = nv;
  dv->vote_id = c->w_vid.as<uint32_t>();
  dv->proposal_id = c->w_pid.as<uint32_t>();
  dv->timestamp = c->w_ts.as<uint64_t>();
  dv->vote = c->w_vote.as<uint8_t>();
  dv->bytes = wire;
  dv->bytes_len = wire_len;
  dv->field_off = c->w_foff.as<uint64_t>();
  dv->field_len = c->w_flen.as<uint32_t>();
  if (nm) {
    hlc::launch_wire_place(nm, vcount, vbegin, c->w_slab_off.as<uint64_t>(), c->w_slab_len.as<uint32_t>(), dprops,
                           c->w_vrec_off.as<uint64_t>(), c->w_vrec_len.as<uint32_t>(), c->w_vrec_msg.as<uint32_t>(), s);
    if (big)  // messages with more vote records than the walker's slab: walk them again, writing in place
      hlc::launch_wire_walk(1, wire, moff, mlen, nm, vcount, vbegin, dwout, dprops, scope, n_scope, nullptr, nullptr,
                            nullptr, c->w_vrec_off.as<uint64_t>(), c->w_vrec_len.as<uint32_t>(),
                            c->w_vrec_msg.as<uint32_t>(), c->w_huge.as<uint64_t>(), s);
    for (uint64_t i = 0, hb = 0; 2 * i < huge.size(); hb += huge[2 * i + 1] / 2 + 1, ++i)
      hlc::launch_huge_place(huge[2 * i], vcount, vbegin, c->h_off.as<uint64_t>() + hb, c->h_len.as<uint32_t>() + hb,
                             c->w_vrec_off.as<uint64_t>(), c->w_vrec_len.as<uint32_t>(),
                             c->w_vrec_msg.as<uint32_t>(), s);
    HIPCHK(hipMemsetAsync(c->w_first_bad.p, 0xFF, nm * 4, s));
    hlc::launch_wire_votes(wire, moff, mlen, nv, c->w_vrec_off.as<uint64_t>(), c->w_vrec_len.as<uint32_t>(),
                           c->w_vrec_msg.as<uint32_t>(), vbegin, dv, c->w_vote_err.as<uint8_t>(),
                           c->w_first_bad.as<uint32_t>(), s);
    hlc::launch_wire_final(nm, vbegin, c->w_vote_err.as<uint8_t>(), c->w_first_bad.as<uint32_t>(), dwout, dprops, s);
  }
  HIPCHK(hipGetLastError());
  *n_votes = nv;
  return 0;
}

int check_wire_host(const uint8_t* wire, uint64_t wire_len, const uint64_t* moff, const uint32_t* mlen, uint64_t nm,
                    const hlc_scope_config* scope, uint64_t n_scope) {
  if (nm && (!moff || !mlen || !scope)) return set_err(HLC_EINVAL, "NULL message / scope array");
  if (nm && n_scope != 1 && n_scope != nm) return set_err(HLC_EINVAL, "n_scope must be 1 or n_msgs");
  for (uint64_t i = 0; i < nm; ++i) {
    if (mlen[i] && (!wire || moff[i] + mlen[i] > wire_len || moff[i] + mlen[i] < moff[i]))
      return set_err(HLC_EINVAL, "message (offset, length) outside the wire buffer");
  }
  return 0;
}

// Stages the wire inputs on the device.
int stage_wire(hlc_ctx* c, const uint8_t* wire, uint64_t wire_len, const uint64_t* moff, const uint32_t* mlen,
               uint64_t nm, const hlc_scope_config* scope, uint64_t n_scope, hipStream_t s) {
  CHK(upload(c->w_wire, wire, wire ? wire_len : 0, s));
  CHK(upload(c->w_moff, moff, nm, s));
  CHK(upload(c->w_mlen, mlen, nm, s));
  CHK(upload(c->w_scope, scope, nm ? n_scope : 0, s));
  CHK(c->w_props.ensure(nm * sizeof(hlc_proposal) + 16));
  CHK(c->w_wout.ensure(nm * sizeof(hlc_wire_proposal) + 16));
  return 0;
}

int check_votes_host(const hlc_votes* v) {
  if (!v) return set_err(HLC_EINVAL, "votes is NULL");
  if (v->n && (!v->vote_id || !v->proposal_id || !v->timestamp || !v->vote || !v->field_off || !v->field_len))
    return set_err(HLC_EINVAL, "NULL vote array");
  for (uint64_t i = 0; i < v->n * HLC_NFIELDS; ++i) {
    if (v->field_len[i] && (!v->bytes || v->field_off[i] + v->field_len[i] > v->bytes_len ||
                            v->field_off[i] + v->field_len[i] < v->field_off[i]))
      return set_err(HLC_EINVAL, "field (offset, length) outside the byte arena");
  }
  return 0;
}

// A caller-side scheme's verdicts (the *_verdicts entries): HLC_VERIFY_TRUE / _FALSE / Err up to HLC_VERIFY_ERR
int check_verdicts(const uint8_t* verdicts, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i)
    if (verdicts[i] > HLC_VERIFY_ERR)
      return set_err(HLC_EINVAL, "verdict " + std::to_string(verdicts[i]) + " at vote " + std::to_string(i) +
                                     " above HLC_VERIFY_ERR");
  return 0;
}

// Stage host votes on the device; returns a device-pointer view in *dv.
int stage_votes(hlc_ctx* c, const hlc_votes* v, hlc_votes* dv, hipStream_t s) {
  const uint64_t n = v->n;
  CHK(upload(c->in_vote_id, v->vote_id, n, s));
  CHK(upload(c->in_pid, v->proposal_id, n, s));
  CHK(upload(c->in_ts, v->timestamp, n, s));
  CHK(upload(c->in_vote, v->vote, n, s));
  CHK(upload(c->in_off, v->field_off, n * HLC_NFIELDS, s));
  CHK(upload(c->in_len, v->field_len, n * HLC_NFIELDS, s));
  CHK(upload(c->in_bytes, v->bytes, v->bytes ? v->bytes_len : 0, s));
  dv->n = n;
  dv->vote_id = c->in_vote_id.as<uint32_t>();
  dv->proposal_id = c->in_pid.as<uint32_t>();
  dv->timestamp = c->in_ts.as<uint64_t>();
  dv->vote = c->in_vote.as<uint8_t>();
  dv->field_off = c->in_off.as<uint64_t>();
  dv->field_len = c->in_len.as<uint32_t>();
  dv->bytes = c->in_bytes.as<uint8_t>();
  dv->bytes_len = v->bytes_len;
  return 0;
}

void destroy_ctx(hlc_ctx* ctx) {
  if (!ctx) return;
  for (hipStream_t x : {ctx->stream, ctx->aux, ctx->aux2, ctx->copy, ctx->dec, ctx->wlk})
    if (x) (void)hipStreamSynchronize(x);
  hipStream_t s = ctx->stream, a = ctx->aux, a2 = ctx->aux2, cp = ctx->copy, dc = ctx->dec, wk = ctx->wlk;
  delete ctx;
  for (hipStream_t x : {s, a, a2, cp, dc, wk})
    if (x) (void)hipStreamDestroy(x);
}

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// The NUMA node of HIP device `device` (sysfs: the device's PCI address -> numa_node), or -1.
int device_node(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  for (char* q = bus; *q; ++q) *q = (char)std::tolower((unsigned char)*q);
  int node = -1;
  std::FILE* f = std::fopen((std::string("/sys/bus/pci/devices/") + bus + "/numa_node").c_str(), "r");
  if (!f) return -1;
  if (std::fscanf(f, "%d", &node) != 1) node = -1;
  std::fclose(f);
  return node;
}

// The node most of the sampled pages of [p, p + len) are on (move_pages without a target: a query,
// nothing moves), or -1 when unknown (not yet touched, or the call is refused).
int memory_node(const void* p, size_t len) {
  if (!p || !len) return -1;
  const uintptr_t page = 4096, a = (uintptr_t)p & ~(page - 1), b = ((uintptr_t)p + len - 1) & ~(page - 1);
  const uint64_t pages = (b - a) / page + 1, k = std::min<uint64_t>(pages, 16);
  void* addr[16];
  int status[16];
  for (uint64_t j = 0; j < k; ++j) addr[j] = reinterpret_cast<void*>(a + page * (k > 1 ? (pages - 1) * j / (k - 1) : 0));
  if (syscall(SYS_move_pages, 0, (unsigned long)k, addr, nullptr, status, 0) != 0) return -1;
  int votes[64] = {0}, best = -1;
  for (uint64_t j = 0; j < k; ++j)
    if (status[j] >= 0 && status[j] < 64 && ++votes[status[j]] > (best >= 0 ? votes[best] : 0)) best = status[j];
  return best;
}

// The CPUs of NUMA node `node` that this process may run on (the node's cpulist intersected with the
// affinity mask), or {} when unknown.
std::vector<int> node_cpus(int node) {
  std::vector<int> out;
  if (node < 0) return out;
  std::FILE* f = std::fopen(("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist").c_str(), "r");
  if (!f) return out;
  char buf[4096] = {0};
  const size_t got = std::fread(buf, 1, sizeof buf - 1, f);
  std::fclose(f);
  buf[got] = 0;
  cpu_set_t aff;
  CPU_ZERO(&aff);
  if (sched_getaffinity(0, sizeof aff, &aff) != 0) return out;
  for (char* q = buf; *q;) {  // "0-63,128-191"
    char* end = nullptr;
    const long a = std::strtol(q, &end, 10);
    if (end == q) break;
    long b = a;
    q = end;
    if (*q == '-') b = std::strtol(q + 1, &q, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET((int)c, &aff)) out.push_back((int)c);
    while (*q == ',' || *q == '\n' || *q == ' ') ++q;
  }
  return out;
}

// The recovery ranges of a host-buffer call of n items (HLC_OPT_SPLIT_VOTES: the first range; the
// environment's HLC_SPLIT_VOTES="a,b,..." a list; default "98304,196608"; 0 = one range): a range of
// each listed size while at least twice that many
// items remain, then ranges of twice the previous size on the same rule (a large batch keeps the
// device busy while the host gathers the next range's signatures; at most 16 ranges), then one
// range for the rest.  Range k's k_rec_main grid starts once its signatures
// have landed; ranges alternate between two streams (and two per-lane scratch buffers), so each
// range's waves take the SIMD slots the previous range's waves free.
std::vector<uint64_t> split_ranges(uint64_t n, const std::vector<uint64_t>& sizes) {
  std::vector<uint64_t> b{0};
  uint64_t x = 0;
  for (size_t k = 0; k < 15; ++k) {
    x = k < sizes.size() ? sizes[k] : 2 * x;
    if (!x || n - b.back() < 2 * x) break;
    b.push_back(b.back() + x);
  }
  if (n > b.back() || b.size() == 1) b.push_back(n);
  return b;  // range k = [b[k], b[k+1])
}

// Whether [p, p + len) lies in page-locked host memory the device can DMA from directly
// (hlc_host_alloc, hipHostMalloc or hipHostRegister): then the host-buffer entries upload that array
// from the caller's memory and skip its staging copy.  The first and the last byte must be page-locked
// host memory of ONE allocation (the same buffer id): an allocation is contiguous, so the whole range
// is then inside it.  Two page-locked blocks that happen to abut, or a buffer registered in two
// separate parts with pageable memory between them, are staged.
bool pinned_buffer(const void* q, unsigned long long& id) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, q) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: clear the sticky error
    return false;
  }
  if (a.type != hipMemoryTypeHost) return false;
  if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)q) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return true;
}
bool is_pinned(const void* p, size_t len) {
  if (!p || !len) return false;
  unsigned long long a = 0, b = 0;
  if (!pinned_buffer(p, a) || !pinned_buffer(static_cast<const uint8_t*>(p) + len - 1, b)) return false;
  return a == b;
}

// The host-buffer entries' streams, events, staging pool and second recovery slot (on first use).
// The runtime maps a process's streams onto a few hardware queues per priority level
// (GPU_MAX_HW_QUEUES, 4 on the box), and a marker recorded on a stream that shares its queue with
// another stream's kernel completes only after that kernel: measured, the upload stream's last event
// fired when the second k_rec_main ended, 4 ms after its DMA, and the prehash waited for it.  So the
// upload stream takes the greatest priority and the second recovery stream the least: each draws
// its queue from a pool of its own, apart from the normal-priority launch / aux streams.
// The staging pool's workers are bound by HLC_OPT_POOL_BIND: not at all (the default: on two boxes,
// near and far inputs, unbound staging was the fastest arm), to the CPUs of the GPU's NUMA node (their
// copies then write the page-locked buffer from the socket the GPU hangs off; the DMA reads it from
// there), or to those of the node the call's largest input (`src`, its arena) lives on (the copies then
// read the caller's pages locally -- a cross-socket read costs more than a cross-socket write, DESIGN.md
// §5).  A node with fewer usable CPUs than workers is not bound to.
int host_resources(hlc_ctx* c, const void* src = nullptr, size_t src_len = 0) {
  int least = 0, greatest = 0;
  HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  if (!c->copy) HIPCHK(hipStreamCreateWithPriority(&c->copy, hipStreamNonBlocking, greatest));
  if (!c->aux2) HIPCHK(hipStreamCreateWithPriority(&c->aux2, hipStreamNonBlocking, least));
  if (!c->dec) HIPCHK(hipStreamCreateWithPriority(&c->dec, hipStreamNonBlocking, greatest));
  if (!c->wlk) HIPCHK(hipStreamCreateWithPriority(&c->wlk, hipStreamNonBlocking, greatest));
  for (hipEvent_t* e : {&c->ev_rest, &c->ev_done})
    if (!*e) HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  if (!c->pool || c->pool->threads() != c->opt.host_threads) {
    c->pool.reset(new HostPool(c->opt.host_threads - 1));
    c->pool_node = -2;
  }
  {
    int node = -1;
    if (c->opt.pool_bind == HLC_POOL_BIND_GPU) node = device_node(c->device);
    else if (c->opt.pool_bind == HLC_POOL_BIND_SOURCE) node = memory_node(src, src_len);
    if (node != c->pool_node) {  // sysfs reads and the rebinding: only when the node changes
      std::vector<int> cpus = node_cpus(node);
      if ((int)cpus.size() < c->opt.host_threads - 1) cpus.clear();
      c->pool->rebind(cpus);
      c->pool_cpus = cpus;
      c->pool_node = node;
    }
  }
  CHK(ensure_recover_scratch(c));
  CHK(c->rec_scratch2.ensure(c->rec_lanes * hlc::recover_scratch_words() * sizeof(uint32_t)));
  return 0;
}

// HLC_HOST_TRACE=1: one line per host-buffer call (hlc_validate_proposals, hlc_validate_wire_proposals,
// hlc_eth_verify_batch) on stderr -- host phase ends and device event times, ms from the call's start
// (the device times from an event recorded first on the upload stream); HLC_HOST_TRACE=2: the same
// JSON kept for hlc_ctx_last_host_trace only (bench.py's per-phase figures), nothing printed.
struct HostTrace {
  using clk = std::chrono::steady_clock;
  bool on = false, print = false;  // HLC_OPT_HOST_TRACE 1: print + keep, 2: keep
  std::string* sink = nullptr;
  clk::time_point t0;
  std::vector<std::pair<std::string, double>> host, facts;
  std::vector<std::pair<std::string, hipEvent_t>> dev;
  hipEvent_t e0 = nullptr;
  // a value about the call (not a time): which inputs were DMA'd from the caller's page-locked memory
  void fact(const std::string& what, double v) {
    if (on) facts.emplace_back(what, v);
  }
  HostTrace(std::string* keep, int level) : on(level != 0), print(level == 1), sink(keep) {
    if (sink) sink->clear();  // hlc_ctx_last_host_trace: "" after a call made without tracing
  }
  void start(hipStream_t s) {
    if (!on) return;
    t0 = clk::now();
    (void)hipEventCreate(&e0);
    (void)hipEventRecord(e0, s);
  }
  void mark(const std::string& what) {
    if (on) host.emplace_back(what, std::chrono::duration<double, std::milli>(clk::now() - t0).count());
  }
  void ev(const std::string& what, hipStream_t s) {
    if (!on) return;
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) == hipSuccess) {
      (void)hipEventRecord(e, s);
      dev.emplace_back(what, e);
    }
  }
  ~HostTrace() {
    if (!on) return;
    (void)hipDeviceSynchronize();
    std::string j = "{\"host\": {";
    char b[96];
    for (size_t k = 0; k < host.size(); ++k) {
      std::snprintf(b, sizeof b, "%s\"%s\": %.3f", k ? ", " : "", host[k].first.c_str(), host[k].second);
      j += b;
    }
    j += "}, \"device\": {";
    for (size_t k = 0; k < dev.size(); ++k) {
      float f = -1;
      (void)hipEventElapsedTime(&f, e0, dev[k].second);
      std::snprintf(b, sizeof b, "%s\"%s\": %.3f", k ? ", " : "", dev[k].first.c_str(), (double)f);
      j += b;
      (void)hipEventDestroy(dev[k].second);
    }
    j += "}, \"facts\": {";
    for (size_t k = 0; k < facts.size(); ++k) {
      std::snprintf(b, sizeof b, "%s\"%s\": %.17g", k ? ", " : "", facts[k].first.c_str(), facts[k].second);
      j += b;
    }
    j += "}}";
    if (print) std::fprintf(stderr, "HLC_HOST_TRACE %s\n", j.c_str());
    if (sink) *sink = j;
    if (e0) (void)hipEventDestroy(e0);
  }
};

// One call's page-locked staging buffer P, its device copy D and the upload stream.
struct Staging {
  hlc_ctx* c;
  uint8_t* P;
  uint8_t* D;
  bool nt = false;  // non-temporal staging copies (HLC_OPT_NT_COPY on a CPU with AVX2)
  int up(size_t off, size_t len) {
    if (len) HIPCHK(hipMemcpyAsync(D + off, P + off, len, hipMemcpyHostToDevice, c->copy));
    return 0;
  }
  // len bytes from the caller's page-locked memory straight to D + off (no staging copy)
  int up_from(size_t off, const void* src, size_t len) {
    if (len) HIPCHK(hipMemcpyAsync(D + off, src, len, hipMemcpyHostToDevice, c->copy));
    return 0;
  }
  void drain() {
    for (hipStream_t x : {c->copy, c->wlk, c->dec, c->aux, c->aux2, c->stream})
      if (x) (void)hipStreamSynchronize(x);
  }
};

// Drains a host-buffer call's streams when it returns early (HLC_EINVAL from a field check, or a HIP
// failure) with work in flight: no upload may still read the page-locked staging buffer, and no range
// kernel may still use the call's workspace or events, when the next call reuses them.
// Disarmed once the call has waited for its outputs.
struct DrainOnExit {
  Staging& st;
  bool armed = true;
  ~DrainOnExit() {
    if (armed) st.drain();
  }
};

// The recovery ranges of a host-buffer call (split_ranges) with their per-vote records and events.
int prepare_ranges(hlc_ctx* c, uint64_t n, std::vector<uint64_t>& rb) {
  rb = split_ranges(n, c->opt.split_votes);
  const size_t R = rb.size() - 1;
  CHK(c->rec_work.ensure(hlc::recover_work_words(n) * sizeof(uint32_t)));
  while (c->rec_works.size() < R) c->rec_works.emplace_back(new DBuf());
  while (c->ev_up.size() < R) {
    hipEvent_t a = nullptr, b = nullptr;
    HIPCHK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
    c->ev_up.push_back(a);
    HIPCHK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
    c->ev_main.push_back(b);
  }
  while (c->ev_prepk.size() < R) {
    hipEvent_t p = nullptr;
    HIPCHK(hipEventCreateWithFlags(&p, hipEventDisableTiming));
    c->ev_prepk.push_back(p);
  }
  for (size_t k = 0; k < R; ++k) CHK(c->rec_works[k]->ensure(hlc::recover_range_words(rb[k + 1] - rb[k]) * 4));
  return 0;
}

// votes per k_rec_prep lane in the first recovery range: HLC_OPT_FIRST_BATCH, default 1 (8 = as the rest)

// Range k's front half of the recovery -- k_rec_prep + k_rec_main over its m items, signatures read
// through (sig_off, sig_len) from the device arena -- on the aux streams in turn (k even: aux, odd:
// aux2, each with its own per-lane scratch), once its upload (ev_up[k]) has landed.
int launch_front(hlc_ctx* c, HostTrace& tr, uint64_t n, size_t k, uint64_t a0, uint64_t m, const uint8_t* dbytes,
                 const uint64_t* sig_off, size_t off_stride, const uint32_t* sig_len, size_t len_stride,
                 std::vector<RecFront>& fronts, hipEvent_t ready = nullptr, uint64_t cap_waves = 0) {
  if (!m) return 0;
  // cap_waves != 0: this range's grid holds at most that many waves (wire_front_cap)
  const uint64_t lanes = cap_waves ? std::min<uint64_t>(c->rec_lanes, cap_waves * 64) : c->rec_lanes;
  // the first range's prep is on the call's critical path with the device otherwise idle: one vote
  // per lane (no batched inversion), so its dependent chain is an eighth as long
  const hlc::RecRange range{a0, m, c->rec_works[k]->as<uint32_t>(), k == 0 ? c->opt.first_batch : 0};
  const bool odd = k % 2;
  hipStream_t a = odd ? c->aux2 : c->aux;
  uint32_t* scratch = (odd ? c->rec_scratch2 : c->rec_scratch).as<uint32_t>();
  HIPCHK(hipStreamWaitEvent(a, ready ? ready : c->ev_up[k], 0));
  hlc::launch_recover_prep(n, dbytes, sig_off, off_stride, sig_len, len_stride, c->rec_work.as<uint32_t>(), a,
                           nullptr, &range);
  HIPCHK(hipEventRecord(c->ev_prepk[k], a));
  hlc::launch_recover_main(n, dbytes, sig_off, off_stride, scratch, lanes, c->rec_work.as<uint32_t>(), a,
                           c->opt.rec_force_exact, &range);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev_main[k], a));
  tr.ev("main_end_" + std::to_string(k), a);
  fronts.push_back(RecFront{a0, a0 + m, c->ev_main[k], c->ev_prepk[k]});
  return 0;
}

// One input array of a host-buffer call: `elem` bytes per item at `src`, staged at `dst`; uploaded
// from the caller's memory when that is page-locked.
struct Arr {
  const uint8_t* src;
  size_t dst, elem;
  bool pinned;
};

// Items [a0, a1) of the arrays: staging copies of the pageable ones (and per part, `also`(part,
// b0, b1) right after its copies, while the rows are in cache: the callers' field checks), then the
// uploads (the pinned ones straight from the caller).
int stage_rows(Staging& st, HostPool& pool, Arr* arr, int na, uint64_t a0, uint64_t a1,
               const std::function<void(int, uint64_t, uint64_t)>& also = nullptr) {
  pool.run([&](int t, int T) {
    const uint64_t b0 = a0 + (a1 - a0) * t / T, b1 = a0 + (a1 - a0) * (t + 1) / T;
    for (int q = 0; q < na; ++q)
      if (!arr[q].pinned && b1 > b0)
        stage_copy(st.P + arr[q].dst + arr[q].elem * b0, arr[q].src + arr[q].elem * b0, arr[q].elem * (b1 - b0),
                   st.nt);
    if (also) also(t, b0, b1);
  });
  for (int q = 0; q < na; ++q) {
    const size_t off = arr[q].elem * a0, len = arr[q].elem * (a1 - a0);
    if (arr[q].pinned) CHK(st.up_from(arr[q].dst + off, arr[q].src + off, len));
    else CHK(st.up(arr[q].dst + off, len));
  }
  return 0;
}

// The arena bytes [lo, hi) (staged unless page-locked) -> the device arena at o_arena.
int stage_span(Staging& st, HostPool& pool, const uint8_t* bytes, bool pinned, size_t o_arena, uint64_t lo,
               uint64_t hi) {
  if (hi <= lo) return 0;
  if (pinned) return st.up_from(o_arena + lo, bytes + lo, hi - lo);
  pool.run([&](int t, int T) {
    const uint64_t d0 = lo + (hi - lo) * t / T, d1 = lo + (hi - lo) * (t + 1) / T;
    if (d1 > d0) stage_copy(st.P + o_arena + d0, bytes + d0, d1 - d0, st.nt);
  });
  return st.up(o_arena + lo, hi - lo);
}

// Pieces the inputs other than the signatures are staged and uploaded in: HLC_OPT_REST_PIECES (default
// 3): piece k+1 is copied into page-locked memory while piece k's DMA runs.

// The signatures of items [a0, a1) (sig_off / sig_len with stride `stride`) gathered by the host
// pool into the dense staging array at o_sig (65 B per item; slots of other lengths left as they
// are) and their lengths at o_len, then uploaded.  false (nothing read) when a 65-byte signature
// lies outside the arena.
bool stage_sigs(Staging& st, HostPool& pool, const uint8_t* bytes, uint64_t bytes_len, const uint64_t* sig_off,
                const uint32_t* sig_len, size_t stride, size_t o_sig, size_t o_len, uint64_t a0, uint64_t a1,
                int* rc) {
  const uint64_t m = a1 - a0;
  std::vector<int> bad(pool.chunks(), 0);
  pool.run([&](int t, int T) {
    const uint64_t b0 = a0 + m * t / T, b1 = a0 + m * (t + 1) / T;
    uint8_t* sg = st.P + o_sig;
    uint32_t* sl = reinterpret_cast<uint32_t*>(st.P + o_len);
    for (uint64_t i = b0; i < b1; ++i) {
      const uint64_t off = sig_off[i * stride];
      const uint32_t len = sig_len[i * stride];
      sl[i] = len;
      if (len != 65) continue;  // the prep stage skips it (a length error decided elsewhere)
      if (!bytes || off + 65 > bytes_len || off + 65 < off) {
        bad[t] = 1;
        return;
      }
      std::memcpy(sg + 65 * i, bytes + off, 65);
    }
  });
  for (int x : bad)
    if (x) return false;
  *rc = st.up(o_sig + 65 * a0, 65 * m);
  if (*rc == 0) *rc = st.up(o_len + 4 * a0, 4 * m);
  return true;
}

// hlc_validate_proposals over host buffers (what INTEGRATION.md's process_incoming_proposals calls).
// The caller's votes go to the device through page-locked staging on the context's upload stream,
// ordered by what the kernels need first, so that the VALU-bound recovery starts long before the
// whole batch has landed:
//   1. per recovery range of split_ranges(n) (growing sizes), the votes' signatures gathered
//      into a dense array (65 B per vote) with their lengths; behind each range's upload, its
//      k_rec_prep + k_rec_main on the two aux streams in turn (each with its own per-lane scratch),
//      so range k's grid waves take the SIMD slots range k-1's waves free (the ranges' grid tails
//      overlap the next range's work), and every range's signatures are on the device after ~69 B
//      per vote of DMA;
//   2. every other input (SoA arrays, proposals, the byte arena) in rest_pieces() pieces, each
//      copied into page-locked memory by the host pool (every field's (offset, length) checked on
//      the way) while the previous piece's DMA runs -> once they have landed, the prehash, chain /
//      duplicate / YES kernels on the launch stream, one recovery finish (u1 G, Z^-1, address) after
//      the last main stage, the statuses, tables, finalize, and one D2H of every output into
//      page-locked memory.
// An array the caller holds in page-locked memory (hlc_host_alloc) is uploaded straight from there
// (the signatures are still gathered).  A field outside the arena returns HLC_EINVAL before any
// kernel that reads it is enqueued and before anything reaches the caller's outputs (the recovery
// ranges already in flight are drained and discarded).  Only
// stream / event dependencies order the stages: no kernel waits on a flag, so any mapping of the
// streams onto hardware queues is correct (one that serialises them is only slower).
int validate_host(hlc_ctx* c, const hlc_votes* v, const hlc_proposal* props, uint64_t np, uint64_t now,
                  hlc_result* out_res, uint8_t* out_st, uint8_t* out_rs, uint8_t* out_rec) {
  const uint64_t n = v->n;
  const uint64_t blen = v->bytes ? v->bytes_len : 0;
  CHK(host_resources(c, v->bytes, blen));
  HostPool& pool = *c->pool;
  HostTrace tr(&c->last_trace, c->opt.host_trace);
  tr.start(c->copy);
  // inputs, page-locked and on the device alike: dense signatures | signature lengths | vote_id |
  // proposal_id | timestamp | vote | field_off | field_len | proposals | arena
  size_t o[11];
  o[0] = 0;
  o[1] = o[0] + al256(n * 65);
  o[2] = o[1] + al256(n * 4);
  o[3] = o[2] + al256(n * 4);
  o[4] = o[3] + al256(n * 4);
  o[5] = o[4] + al256(n * 8);
  o[6] = o[5] + al256(n);
  o[7] = o[6] + al256(n * 8 * HLC_NFIELDS);
  o[8] = o[7] + al256(n * 4 * HLC_NFIELDS);
  o[9] = o[8] + al256(np * sizeof(hlc_proposal));
  o[10] = o[9] + blen;
  // outputs: results | status | reason | recovered
  size_t r[5];
  r[0] = 0;
  r[1] = al256((np + 1) * sizeof(hlc_result));
  r[2] = r[1] + al256(n + 1);
  r[3] = r[2] + al256(n + 1);
  r[4] = r[3] + (out_rec ? al256(n * 20 + 20) : 0);
  CHK(c->pin_in.ensure(o[10] + 16));
  CHK(c->dev_in.ensure(o[10] + 16));
  CHK(c->pin_out.ensure(r[4] + 16));
  CHK(c->dev_out.ensure(r[4] + 16));
  CHK(reserve_validate(c, n, np));
  std::vector<uint64_t> rb;
  CHK(prepare_ranges(c, n, rb));
  Staging st{c, c->pin_in.at(0), c->dev_in.as<uint8_t>(), c->opt.nt_copy && cpu_has_avx2()};
  DrainOnExit guard{st};
  const uint8_t* D = st.D;
  const int parts = pool.chunks();
  std::vector<RecFront> fronts;
  for (size_t k = 0; k + 1 < rb.size(); ++k) {
    const uint64_t a0 = rb[k], a1 = rb[k + 1];
    int rc = 0;
    if (!stage_sigs(st, pool, v->bytes, v->bytes_len, v->field_off + HLC_F_SIGNATURE, v->field_len + HLC_F_SIGNATURE,
                    HLC_NFIELDS, o[0], o[1], a0, a1, &rc))
      return set_err(HLC_EINVAL, "field (offset, length) outside the byte arena");
    CHK(rc);
    HIPCHK(hipEventRecord(c->ev_up[k], c->copy));
    tr.mark("sigs_staged_" + std::to_string(k));
    tr.ev("sigs_landed_" + std::to_string(k), c->copy);
    CHK(launch_front(c, tr, n, k, a0, a1 - a0, D + o[0] + 65 * a0, nullptr, 0,
                     reinterpret_cast<const uint32_t*>(D + o[1]) + a0, 1, fronts));
  }
  // everything else, piece by piece; the field checks ride along with the rows' staging copies
  Arr arr[6] = {{reinterpret_cast<const uint8_t*>(v->vote_id), o[2], 4, false},
                {reinterpret_cast<const uint8_t*>(v->proposal_id), o[3], 4, false},
                {reinterpret_cast<const uint8_t*>(v->timestamp), o[4], 8, false},
                {v->vote, o[5], 1, false},
                {reinterpret_cast<const uint8_t*>(v->field_off), o[6], 8 * HLC_NFIELDS, false},
                {reinterpret_cast<const uint8_t*>(v->field_len), o[7], 4 * HLC_NFIELDS, false}};
  for (Arr& x : arr) x.pinned = is_pinned(x.src, x.elem * n);
  Arr parr{reinterpret_cast<const uint8_t*>(props), o[8], sizeof(hlc_proposal), false};
  parr.pinned = is_pinned(props, np * sizeof(hlc_proposal));
  const bool arena_pinned = is_pinned(v->bytes, blen);
  {  // bit q: arr[q] DMA'd straight from the caller (vote_id, proposal_id, timestamp, vote, field_off,
     // field_len), bit 6: the proposals, bit 7: the arena
    int mask = 0;
    for (int q = 0; q < 6; ++q) mask |= arr[q].pinned ? 1 << q : 0;
    tr.fact("pinned_mask", mask | (parr.pinned ? 64 : 0) | (arena_pinned ? 128 : 0));
    tr.fact("pool_cpus", (double)c->pool_cpus.size());
    if (tr.on) {  // NUMA placement of the call: the arena, the staging buffer, the workers' node, the GPU's
      tr.fact("arena_node", memory_node(v->bytes, blen));
      tr.fact("staging_node", memory_node(st.P, o[10]));
      tr.fact("pool_node", c->pool_node);
      tr.fact("gpu_node", device_node(c->device));
    }
  }
  CHK(stage_rows(st, pool, &parr, 1, 0, np));
  std::vector<int> bad(parts, 0);
  const int K = c->opt.rest_pieces;
  for (int k = 0; k < K; ++k) {
    const uint64_t v0 = n * k / K, v1 = n * (k + 1) / K;
    CHK(stage_rows(st, pool, arr, 6, v0, v1, [&](int t, uint64_t b0, uint64_t b1) {
      for (uint64_t i = b0 * HLC_NFIELDS; i < b1 * HLC_NFIELDS; ++i) {
        const uint64_t off = v->field_off[i], len = v->field_len[i];
        if (len && (!v->bytes || off + len > v->bytes_len || off + len < off)) {
          bad[t] = 1;
          return;
        }
      }
    }));
    CHK(stage_span(st, pool, v->bytes, arena_pinned, o[9], blen * k / K, blen * (k + 1) / K));
  }
  // a field outside the arena: nothing that reads the fields is enqueued (the recovery ranges
  // already in flight read only the signatures, checked when they were gathered)
  for (int x : bad)
    if (x) return set_err(HLC_EINVAL, "field (offset, length) outside the byte arena");
  tr.mark("rest_staged");
  HIPCHK(hipEventRecord(c->ev_rest, c->copy));
  tr.ev("rest_landed", c->copy);
  // the validation on the launch stream, the recovery ranges joined in by their events
  hipStream_t s = c->stream;
  HIPCHK(hipStreamWaitEvent(s, c->ev_rest, 0));
  hlc_votes dv;
  dv.n = n;
  dv.vote_id = reinterpret_cast<const uint32_t*>(D + o[2]);
  dv.proposal_id = reinterpret_cast<const uint32_t*>(D + o[3]);
  dv.timestamp = reinterpret_cast<const uint64_t*>(D + o[4]);
  dv.vote = D + o[5];
  dv.field_off = reinterpret_cast<const uint64_t*>(D + o[6]);
  dv.field_len = reinterpret_cast<const uint32_t*>(D + o[7]);
  dv.bytes = D + o[9];
  dv.bytes_len = blen;
  uint8_t* ob = c->dev_out.as<uint8_t>();
  CHK(validate_device(c, &dv, reinterpret_cast<const hlc_proposal*>(D + o[8]), np, now,
                      reinterpret_cast<hlc_result*>(ob + r[0]), ob + r[1], ob + r[2], out_rec ? ob + r[3] : nullptr, s,
                      fronts.data(), (int)fronts.size()));
  tr.ev("kernels_end", s);
  HIPCHK(hipMemcpyAsync(c->pin_out.p, ob, r[4], hipMemcpyDeviceToHost, s));
  HIPCHK(hipEventRecord(c->ev_done, s));
  tr.ev("outputs_landed", s);
  tr.mark("enqueued");
  HIPCHK(hipEventSynchronize(c->ev_done));
  guard.armed = false;
  tr.mark("device_done");
  const uint8_t* src = c->pin_out.at(0);
  pool.run([&](int t, int T) {
    const uint64_t b0 = np * t / T, b1 = np * (t + 1) / T, a0 = n * t / T, a1 = n * (t + 1) / T;
    if (b1 > b0) std::memcpy(out_res + b0, src + r[0] + b0 * sizeof(hlc_result), (b1 - b0) * sizeof(hlc_result));
    if (a1 > a0) {
      if (out_st) std::memcpy(out_st + a0, src + r[1] + a0, a1 - a0);
      if (out_rs) std::memcpy(out_rs + a0, src + r[2] + a0, a1 - a0);
      if (out_rec) std::memcpy(out_rec + 20 * a0, src + r[3] + 20 * a0, 20 * (a1 - a0));
    }
  });
  tr.mark("outputs_copied");
  return 0;
}

// hlc_eth_verify_batch over host buffers: the same schedule as validate_host -- the signatures
// first (dense, per recovery range, each range's k_rec_prep + k_rec_main behind its upload on the aux
// streams in turn), then the per-item offsets / lengths and the arena in pieces, field checks on the
// way -- with the verify byte stage (length checks + EIP-191 keccak of each payload, k_verify_prehash)
// on the launch stream once they have landed, each range's finish after its main stage, one D2H of
// the statuses (and addresses).  An (offset, length) outside the arena returns HLC_EINVAL before
// anything reaches the caller's outputs.
int verify_host(hlc_ctx* c, uint64_t n, const uint8_t* bytes, uint64_t bytes_len, const uint64_t* id_off,
                const uint32_t* id_len, const uint64_t* pay_off, const uint32_t* pay_len, const uint64_t* sig_off,
                const uint32_t* sig_len, uint8_t* out_status, uint8_t* out_addr) {
  const uint64_t blen = bytes ? bytes_len : 0;
  CHK(host_resources(c, bytes, blen));
  HostPool& pool = *c->pool;
  HostTrace tr(&c->last_trace, c->opt.host_trace);
  tr.start(c->copy);
  // inputs: dense signatures | signature lengths | identity / payload lengths | identity / payload
  // offsets | arena
  size_t o[8];
  o[0] = 0;
  o[1] = o[0] + al256(n * 65);
  o[2] = o[1] + al256(n * 4);
  o[3] = o[2] + al256(n * 4);
  o[4] = o[3] + al256(n * 4);
  o[5] = o[4] + al256(n * 8);
  o[6] = o[5] + al256(n * 8);
  o[7] = o[6] + blen;
  const size_t r1 = al256(n + 1), r2 = r1 + (out_addr ? al256(n * 20) : 0);  // statuses | addresses
  CHK(c->pin_in.ensure(o[7] + 16));
  CHK(c->dev_in.ensure(o[7] + 16));
  CHK(c->pin_out.ensure(r2 + 16));
  CHK(c->dev_out.ensure(r2 + 16));
  CHK(c->pre.ensure(n + 1));
  CHK(c->kec_dig.ensure(n * 32 + 32));
  std::vector<uint64_t> rb;
  CHK(prepare_ranges(c, n, rb));
  Staging st{c, c->pin_in.at(0), c->dev_in.as<uint8_t>(), c->opt.nt_copy && cpu_has_avx2()};
  DrainOnExit guard{st};
  const uint8_t* D = st.D;
  const int parts = pool.chunks();
  std::vector<RecFront> fronts;
  for (size_t k = 0; k + 1 < rb.size(); ++k) {
    const uint64_t a0 = rb[k], a1 = rb[k + 1];
    int rc = 0;
    if (!stage_sigs(st, pool, bytes, bytes_len, sig_off, sig_len, 1, o[0], o[1], a0, a1, &rc))
      return set_err(HLC_EINVAL, "item (offset, length) outside the byte arena");
    CHK(rc);
    HIPCHK(hipEventRecord(c->ev_up[k], c->copy));
    tr.mark("sigs_staged_" + std::to_string(k));
    tr.ev("sigs_landed_" + std::to_string(k), c->copy);
    CHK(launch_front(c, tr, n, k, a0, a1 - a0, D + o[0] + 65 * a0, nullptr, 0,
                     reinterpret_cast<const uint32_t*>(D + o[1]) + a0, 1, fronts));
  }
  Arr arr[4] = {{reinterpret_cast<const uint8_t*>(id_len), o[2], 4, false},
                {reinterpret_cast<const uint8_t*>(pay_len), o[3], 4, false},
                {reinterpret_cast<const uint8_t*>(id_off), o[4], 8, false},
                {reinterpret_cast<const uint8_t*>(pay_off), o[5], 8, false}};
  for (Arr& x : arr) x.pinned = is_pinned(x.src, x.elem * n);
  const bool arena_pinned = is_pinned(bytes, blen);
  std::vector<int> bad(parts, 0);
  const int K = c->opt.rest_pieces;
  for (int k = 0; k < K; ++k) {
    const uint64_t v0 = n * k / K, v1 = n * (k + 1) / K;
    CHK(stage_rows(st, pool, arr, 4, v0, v1, [&](int t, uint64_t b0, uint64_t b1) {
      for (uint64_t i = b0; i < b1; ++i) {
        const uint64_t f[3][2] = {{id_off[i], id_len[i]}, {pay_off[i], pay_len[i]}, {sig_off[i], sig_len[i]}};
        for (const auto& x : f) {
          if (x[0] + x[1] > bytes_len || x[0] + x[1] < x[0] || (x[1] && !bytes)) {
            bad[t] = 1;
            return;
          }
        }
      }
    }));
    CHK(stage_span(st, pool, bytes, arena_pinned, o[6], blen * k / K, blen * (k + 1) / K));
  }
  for (int x : bad)  // nothing that reads identities / payloads is enqueued
    if (x) return set_err(HLC_EINVAL, "item (offset, length) outside the byte arena");
  tr.mark("rest_staged");
  HIPCHK(hipEventRecord(c->ev_rest, c->copy));
  tr.ev("rest_landed", c->copy);
  hipStream_t s = c->stream;
  HIPCHK(hipStreamWaitEvent(s, c->ev_rest, 0));
  const uint8_t* dbytes = D + o[6];
  const uint64_t* did_off = reinterpret_cast<const uint64_t*>(D + o[4]);
  uint8_t* ob = c->dev_out.as<uint8_t>();
  uint8_t* dstat = ob;
  uint8_t* daddr = out_addr ? ob + r1 : nullptr;
  hlc::launch_verify_prehash(n, dbytes, reinterpret_cast<const uint64_t*>(D + o[5]),
                             reinterpret_cast<const uint32_t*>(D + o[3]), reinterpret_cast<const uint32_t*>(D + o[1]),
                             reinterpret_cast<const uint32_t*>(D + o[2]), c->kec_dig.as<uint32_t>(),
                             c->pre.as<uint8_t>(), dstat, s);
  if (daddr) HIPCHK(hipMemsetAsync(daddr, 0, n * 20, s));
  for (const RecFront& f : fronts) HIPCHK(hipStreamWaitEvent(s, f.done, 0));
  hlc::launch_recover_finish(n, c->pre.as<uint8_t>(), c->kec_dig.as<uint32_t>(), dbytes, did_off, 1,
                             c->gtab, c->rec_work.as<uint32_t>(), dstat, daddr, s, c->opt.rec_force_exact);
  HIPCHK(hipGetLastError());
  tr.ev("kernels_end", s);
  HIPCHK(hipMemcpyAsync(c->pin_out.p, ob, r2, hipMemcpyDeviceToHost, s));
  HIPCHK(hipEventRecord(c->ev_done, s));
  tr.ev("outputs_landed", s);
  tr.mark("enqueued");
  HIPCHK(hipEventSynchronize(c->ev_done));
  guard.armed = false;
  tr.mark("device_done");
  const uint8_t* src = c->pin_out.at(0);
  pool.run([&](int t, int T) {
    const uint64_t a0 = n * t / T, a1 = n * (t + 1) / T;
    if (a1 > a0) {
      std::memcpy(out_status + a0, src + a0, a1 - a0);
      if (out_addr) std::memcpy(out_addr + 20 * a0, src + r1 + 20 * a0, 20 * (a1 - a0));
    }
  });
  tr.mark("outputs_copied");
  return 0;
}

// hlc_validate_wire_proposals without pipelining: the whole wire buffer uploaded, decoded, validated
// (messages over wire_huge_threshold(), and the fallback of validate_wire_host).
int wire_host_plain(hlc_ctx* c, const uint8_t* wire, uint64_t wire_len, const uint64_t* moff, const uint32_t* mlen,
                    uint64_t nm, const hlc_scope_config* scope, uint64_t n_scope, uint64_t now, hlc_result* out_res,
                    hlc_wire_proposal* out_wire, uint64_t* out_n_votes) {
  hipStream_t s = c->stream;
  CHK(stage_wire(c, wire, wire_len, moff, mlen, nm, scope, n_scope, s));
  CHK(c->w_res.ensure(nm * sizeof(hlc_result) + 16));
  hlc_votes dv;
  uint64_t nv = 0;
  CHK(decode_device(c, c->w_wire.as<uint8_t>(), wire_len, c->w_moff.as<uint64_t>(), c->w_mlen.as<uint32_t>(), nm,
                    c->w_scope.as<hlc_scope_config>(), n_scope, c->w_props.as<hlc_proposal>(),
                    c->w_wout.as<hlc_wire_proposal>(), &dv, &nv, s));
  CHK(validate_device(c, &dv, c->w_props.as<hlc_proposal>(), nm, now, c->w_res.as<hlc_result>(), nullptr, nullptr,
                      nullptr, s));
  hlc::launch_wire_results(nm, c->w_wout.as<hlc_wire_proposal>(), c->w_res.as<hlc_result>(), s);
  HIPCHK(hipGetLastError());
  if (nm) {
    HIPCHK(hipMemcpyAsync(out_res, c->w_res.p, nm * sizeof(hlc_result), hipMemcpyDeviceToHost, s));
    if (out_wire)
      HIPCHK(hipMemcpyAsync(out_wire, c->w_wout.p, nm * sizeof(hlc_wire_proposal), hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  if (out_n_votes) *out_n_votes = nv;
  c->wire_hint = std::max(c->wire_hint, nv);
  return 0;
}

// The message ranges of a pipelined wire call: range k = messages [mb[k], mb[k+1]), which lie in the
// byte prefix [0, ub[k+1]) of the wire buffer (ub[k] = the largest message end among earlier messages;
// range k uploads [ub[k], ub[k+1])).  Byte sizes as split_ranges' vote counts: HLC_WIRE_SPLIT_BYTES
// ("a,b,...", default 8, 16, 24, 32 MiB -- about 45k, 90k, 135k and 180k votes of config 2's 187 B per
// vote), a range of each listed size while at least twice that many bytes remain, then doubling, at
// most 16 ranges, then one range for the rest.  Swept on the box (tools/wire_pipe.py,
// profiles/r05/wire_pipe_sweep.txt): 8,16,24,32 MiB beat 8,16 / 16,32 / 8,16,24 / 4,8,16,24 and a
// shrinking tail (8,16,24,24,16,16,8) by 1-4%.  Messages that are out of order in the buffer only make a
// range's prefix longer (an earlier range may then upload everything).
void wire_ranges(const uint64_t* moff, const uint32_t* mlen, uint64_t nm, std::vector<uint64_t>& mb,
                 std::vector<uint64_t>& ub, const std::vector<uint64_t>& sizes) {
  std::vector<uint64_t> pre(nm);  // prefix maximum of the message ends (empty messages read nothing)
  uint64_t hi = 0;
  for (uint64_t m = 0; m < nm; ++m) {
    if (mlen[m]) hi = std::max(hi, moff[m] + mlen[m]);
    pre[m] = hi;
  }
  mb.assign(1, 0);
  ub.assign(1, 0);
  uint64_t x = 0, m = 0;
  for (size_t k = 0; k < 15 && nm; ++k) {
    x = k < sizes.size() ? sizes[k] : 2 * x;
    if (!x || hi - ub.back() < 2 * x) break;
    while (m < nm && pre[m] < ub.back() + x) ++m;
    if (m + 1 >= nm) break;
    mb.push_back(m + 1);
    ub.push_back(pre[m]);
    ++m;
  }
  if (mb.back() < nm) {
    mb.push_back(nm);
    ub.push_back(hi);
  }
}

// Waves per recovery grid of every message range but the last (HLC_OPT_WIRE_FRONT_CAP, default 1536 of the
// 2,048 a full grid holds; 0 = full grids).  Two overlapping full grids hold every VGPR of the device, so
// the next range's decode and prep wait until one drains (profiles/r05/wire_host_call_timeline.txt);
// capped grids leave them room.  +0.5 to +2.3% from host buffers over four A/B sessions
// (profiles/r05/ab_wire_front_cap.txt); the last range runs alone at the end and keeps the full grid.
// (the option's value; launch_front gives a capped grid at least one block)
//
// Bytes per staging / upload piece of the wire host entry: HLC_OPT_WIRE_CHUNK, default 4 MiB (8 MiB
// measured 1-2% slower with non-temporal staging copies): piece j+1 is copied into page-locked memory
// while piece j's DMA runs.

// hlc_validate_wire_proposals over host buffers, pipelined: gossip bytes go to
// the device in message ranges (wire_ranges), and each range is decoded and its signatures recovered
// as it lands, the way validate_host's signatures-first ranges start the recovery early:
//   1. the message extents and scope configs go up first (12 B + 16 B per message); then the wire
//      bytes, range by range, in wire_chunk() pieces: the host pool copies piece j+1 into page-locked
//      memory while piece j's DMA runs (a page-locked wire buffer is DMA'd straight from the caller);
//   2. behind range k's last piece, on the walk stream (greatest priority): the walker over its
//      messages and one block scanning their vote counts (vote_begin relative to the range) that writes
//      the range's vote total into mapped page-locked memory; the host polls for it between the next
//      range's pieces, so the pieces keep flowing, and the walks of later ranges queue behind their
//      bytes without waiting for the host;
//   3. with the total known, on the decode stream (greatest priority, so its kernels are dispatched
//      ahead of the recovery grids): the range's records placed, its Vote records decoded at vote base
//      b_k (the sum of the earlier ranges' totals; per-message arrays at the range's first message,
//      per-vote arrays at b_k, so the numbering equals a decode of the whole buffer), and its first-
//      error pass; then its k_rec_prep + k_rec_main on the aux streams in turn, reading the signatures
//      through the decoded (offset, length) pairs straight out of the device wire buffer;
//   4. once every range is decoded: the validation over all votes on the launch stream (prehash, chain,
//      duplicate, tally), one recovery finish after the last main stage, and one D2H of the results.
// The per-vote arrays and the recovery records (row stride N) are sized once, after the first range's
// total: N = the whole call's votes estimated from the first range's density (x 1.25, at least the
// largest total an earlier call decoded, at most wire bytes / 2 -- a vote record takes at least a key
// and a length byte).  A call that decodes more than N votes is drained and re-run unpipelined
// (wire_host_plain), as is any call with a message over wire_huge_threshold() (the parallel huge-message
// decoder needs its own host round trips).  Only stream / event dependencies order the device work.
int validate_wire_host(hlc_ctx* c, const uint8_t* wire, uint64_t wire_len, const uint64_t* moff, const uint32_t* mlen,
                       uint64_t nm, const hlc_scope_config* scope, uint64_t n_scope, uint64_t now, hlc_result* out_res,
                       hlc_wire_proposal* out_wire, uint64_t* out_n_votes) {
  bool plain = nm == 0 || !wire;
  for (uint64_t m = 0; m < nm && !plain; ++m) plain = mlen[m] > hlc::wire_huge_threshold();
  if (plain) return wire_host_plain(c, wire, wire_len, moff, mlen, nm, scope, n_scope, now, out_res, out_wire,
                                    out_n_votes);
  CHK(host_resources(c, wire, wire_len));
  HostPool& pool = *c->pool;
  HostTrace tr(&c->last_trace, c->opt.host_trace);
  tr.start(c->copy);
  std::vector<uint64_t> mb, ub;
  wire_ranges(moff, mlen, nm, mb, ub, c->opt.wire_split_bytes);
  const size_t R = mb.size() - 1;
  const uint64_t U = ub.back();
  // page-locked staging and its device copy: message offsets | lengths | scope configs | wire bytes
  // [0, U) (the bytes past the last message end are never read)
  size_t o[5];
  o[0] = 0;
  o[1] = al256(nm * 8);
  o[2] = o[1] + al256(nm * 4);
  o[3] = o[2] + al256(n_scope * sizeof(hlc_scope_config));
  o[4] = o[3] + al256(U + 16);
  CHK(c->pin_in.ensure(o[4] + 16));
  CHK(c->dev_in.ensure(o[4] + 16));
  const size_t r1 = al256(nm * sizeof(hlc_result)), r2 = r1 + nm * sizeof(hlc_wire_proposal);  // results | wire info
  CHK(c->pin_out.ensure(r2 + 16));
  CHK(c->pin_cnt.ensure(R * 32 + 32));
  // per-message device workspace (the per-vote arrays follow the first range's total)
  const uint64_t slab = hlc::wire_slab();
  CHK(c->w_vcount.ensure(nm * 8 + 8));
  CHK(c->w_vbegin.ensure(nm * 8 + 8));
  CHK(c->w_slab_off.ensure(nm * slab * 8 + 8));
  CHK(c->w_slab_len.ensure(nm * slab * 4 + 4));
  CHK(c->w_big.ensure(32));
  CHK(c->w_huge.ensure(nm * 16 + 16));
  CHK(c->w_first_bad.ensure(nm * 4 + 4));
  CHK(c->w_props.ensure(nm * sizeof(hlc_proposal) + 16));
  CHK(c->w_wout.ensure(nm * sizeof(hlc_wire_proposal) + 16));
  CHK(c->w_res.ensure(nm * sizeof(hlc_result) + 16));
  while (c->ev_cnt.size() < R) {
    hipEvent_t a = nullptr, b = nullptr;
    HIPCHK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
    c->ev_cnt.push_back(a);
    HIPCHK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
    c->ev_dec.push_back(b);
  }
  while (c->ev_up.size() < R) {
    hipEvent_t a = nullptr, b = nullptr;
    HIPCHK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
    c->ev_up.push_back(a);
    HIPCHK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
    c->ev_main.push_back(b);
  }
  while (c->ev_prepk.size() < R) {
    hipEvent_t p = nullptr;
    HIPCHK(hipEventCreateWithFlags(&p, hipEventDisableTiming));
    c->ev_prepk.push_back(p);
  }
  while (c->rec_works.size() < R) c->rec_works.emplace_back(new DBuf());
  Staging st{c, c->pin_in.at(0), c->dev_in.as<uint8_t>(), c->opt.nt_copy && cpu_has_avx2()};
  DrainOnExit guard{st};
  uint8_t* D = st.D;
  const uint8_t* dwire = D + o[3];
  const uint64_t* dmoff = reinterpret_cast<const uint64_t*>(D + o[0]);
  const uint32_t* dmlen = reinterpret_cast<const uint32_t*>(D + o[1]);
  const hlc_scope_config* dscope = reinterpret_cast<const hlc_scope_config*>(D + o[2]);
  hipStream_t s = c->stream;
  uint64_t* vcount = c->w_vcount.as<uint64_t>();
  uint64_t* vbegin = c->w_vbegin.as<uint64_t>();
  hlc_proposal* dprops = c->w_props.as<hlc_proposal>();
  hlc_wire_proposal* dwout = c->w_wout.as<hlc_wire_proposal>();
  uint64_t* cnt = reinterpret_cast<uint64_t*>(c->pin_cnt.p);
  // 1. the message extents and scope configs
  std::memcpy(st.P + o[0], moff, nm * 8);
  std::memcpy(st.P + o[1], mlen, nm * 4);
  std::memcpy(st.P + o[2], scope, n_scope * sizeof(hlc_scope_config));
  CHK(st.up(0, o[3]));
  const bool wire_pinned = is_pinned(wire, U);
  const uint64_t chunk = c->opt.wire_chunk;
  const uint64_t front_cap = c->opt.wire_front_cap;
  tr.fact("ranges", (double)R);
  tr.fact("front_cap_waves", (double)front_cap);
  tr.fact("wire_pinned", wire_pinned ? 1 : 0);
  tr.fact("pool_cpus", (double)c->pool_cpus.size());
  uint64_t N = 0, base = 0;  // per-vote capacity (fixed after range 0), votes decoded so far
  size_t walked = 0, done = 0;
  bool overflow = false;
  std::vector<RecFront> fronts;
  hlc_votes dv{};
  // range k's walk + scan + vote total read-back, on the walk stream behind its bytes: two kernels (the
  // walker; one block scanning the counts and writing the total into mapped page-locked memory)
  uint64_t* cnt_dev = nullptr;
  HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&cnt_dev), c->pin_cnt.p, 0));
  hipStream_t ws = c->wlk;
  auto walk = [&](size_t k) -> int {
    const uint64_t m0 = mb[k], mk = mb[k + 1] - m0;
    HIPCHK(hipStreamWaitEvent(ws, c->ev_up[k], 0));
    hlc::launch_wire_walk(0, dwire, dmoff + m0, dmlen + m0, mk, vcount + m0, nullptr, dwout + m0, dprops + m0,
                          n_scope == 1 ? dscope : dscope + m0, n_scope, c->w_slab_off.as<uint64_t>() + m0 * slab,
                          c->w_slab_len.as<uint32_t>() + m0 * slab, c->w_big.as<uint32_t>(), nullptr, nullptr,
                          nullptr, c->w_huge.as<uint64_t>(), ws, c->w_first_bad.as<uint32_t>() + m0,
                          c->opt.wire_walk);
    hlc::launch_wire_range_scan(vcount + m0, vbegin + m0, mk, cnt_dev + 4 * k, ws);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev_cnt[k], ws));
    tr.ev("walked_" + std::to_string(k), ws);
    return 0;
  };
  // the per-vote arrays at capacity n_cap (before any kernel writes them)
  auto size_votes = [&](uint64_t n_cap) -> int {
    CHK(c->w_vrec_off.ensure(n_cap * 8 + 8));
    CHK(c->w_vrec_len.ensure(n_cap * 4 + 4));
    CHK(c->w_vrec_msg.ensure(n_cap * 4 + 4));
    CHK(c->w_vote_err.ensure(n_cap + 1));
    CHK(c->w_vid.ensure(n_cap * 4 + 4));
    CHK(c->w_pid.ensure(n_cap * 4 + 4));
    CHK(c->w_ts.ensure(n_cap * 8 + 8));
    CHK(c->w_vote.ensure(n_cap + 1));
    CHK(c->w_foff.ensure(n_cap * 8 * HLC_NFIELDS + 8));
    CHK(c->w_flen.ensure(n_cap * 4 * HLC_NFIELDS + 4));
    CHK(reserve_validate(c, n_cap, nm));
    CHK(c->rec_work.ensure(hlc::recover_work_words(n_cap) * sizeof(uint32_t)));
    dv.vote_id = c->w_vid.as<uint32_t>();
    dv.proposal_id = c->w_pid.as<uint32_t>();
    dv.timestamp = c->w_ts.as<uint64_t>();
    dv.vote = c->w_vote.as<uint8_t>();
    dv.bytes = dwire;
    dv.bytes_len = wire_len;
    dv.field_off = c->w_foff.as<uint64_t>();
    dv.field_len = c->w_flen.as<uint32_t>();
    return 0;
  };
  // range k once its total is known: records placed, Vote records decoded at vote base `base`, the
  // first-error pass, then its recovery front half
  auto decode = [&](size_t k) -> int {
    const uint64_t m0 = mb[k], mk = mb[k + 1] - m0;
    const uint64_t nv = cnt[4 * k];
    const bool big = cnt[4 * k + 1] != 0;
    if (k == 0) {
      const uint64_t est = (uint64_t)((double)nv * (double)U / (double)std::max<uint64_t>(ub[1], 1) * 1.25) + 4096;
      N = std::min(U / 2 + 1, std::max(est, c->wire_hint));
      N = std::max(N, nv);
      CHK(size_votes(N));
    }
    if (base + nv > N) {
      overflow = true;
      return 0;
    }
    hipStream_t ds = c->dec;  // behind the walk's read-back on the launch stream (already complete)
    HIPCHK(hipStreamWaitEvent(ds, c->ev_cnt[k], 0));
    hlc_votes dk = dv;  // the range's votes
    dk.n = nv;
    dk.vote_id += base;
    dk.proposal_id += base;
    dk.timestamp += base;
    dk.vote += base;
    dk.field_off += base * HLC_NFIELDS;
    dk.field_len += base * HLC_NFIELDS;
    uint64_t* vro = c->w_vrec_off.as<uint64_t>() + base;
    uint32_t* vrl = c->w_vrec_len.as<uint32_t>() + base;
    uint32_t* vrm = c->w_vrec_msg.as<uint32_t>() + base;
    // (first_bad of the range's messages was reset by the walker)
    if (!big) {  // every record in the walker's slab: place + decode in one kernel
      hlc::launch_wire_votes_slab(dwire, dmoff + m0, dmlen + m0, mk, vcount + m0, vbegin + m0,
                                  c->w_slab_off.as<uint64_t>() + m0 * slab, c->w_slab_len.as<uint32_t>() + m0 * slab,
                                  dprops + m0, base, &dk, c->w_vote_err.as<uint8_t>() + base,
                                  c->w_first_bad.as<uint32_t>() + m0, ds);
    } else {
      hlc::launch_wire_place(mk, vcount + m0, vbegin + m0, c->w_slab_off.as<uint64_t>() + m0 * slab,
                             c->w_slab_len.as<uint32_t>() + m0 * slab, dprops + m0, vro, vrl, vrm, ds, base);
      hlc::launch_wire_walk(1, dwire, dmoff + m0, dmlen + m0, mk, vcount + m0, vbegin + m0, dwout + m0, dprops + m0,
                            n_scope == 1 ? dscope : dscope + m0, n_scope, nullptr, nullptr, nullptr, vro, vrl, vrm,
                            c->w_huge.as<uint64_t>(), ds);
      hlc::launch_wire_votes(dwire, dmoff + m0, dmlen + m0, nv, vro, vrl, vrm, vbegin + m0, &dk,
                             c->w_vote_err.as<uint8_t>() + base, c->w_first_bad.as<uint32_t>() + m0, ds);
    }
    HIPCHK(hipGetLastError());
    // the range's recovery needs the decoded signature fields only: it starts here, and the first-error
    // pass (which only marks failed messages) follows on the decode stream
    HIPCHK(hipEventRecord(c->ev_dec[k], ds));
    tr.ev("decoded_" + std::to_string(k), ds);
    hlc::launch_wire_final(mk, vbegin + m0, c->w_vote_err.as<uint8_t>() + base, c->w_first_bad.as<uint32_t>() + m0,
                           dwout + m0, dprops + m0, ds);
    HIPCHK(hipGetLastError());
    if (nv) {
      CHK(c->rec_works[k]->ensure(hlc::recover_range_words(nv) * 4));
      CHK(launch_front(c, tr, N, k, base, nv, dwire, dk.field_off + HLC_F_SIGNATURE, HLC_NFIELDS,
                       dk.field_len + HLC_F_SIGNATURE, HLC_NFIELDS, fronts, c->ev_dec[k], k + 1 < R ? front_cap : 0));
    }
    base += nv;
    return 0;
  };
  // decodes every walked range whose total has come back (all of them when `wait`)
  auto drain_counts = [&](bool wait) -> int {
    while (done < walked && !overflow) {
      if (wait) {
        HIPCHK(hipEventSynchronize(c->ev_cnt[done]));
      } else {
        const hipError_t q = hipEventQuery(c->ev_cnt[done]);
        if (q == hipErrorNotReady) {
          (void)hipGetLastError();  // not an error: the total is still on its way
          return 0;
        }
        HIPCHK(q);
      }
      tr.mark("count_" + std::to_string(done));
      CHK(decode(done));
      ++done;
    }
    return 0;
  };
  // Workspace that a call of this size needed before (wire_hint: the most votes a call on this context
  // decoded) is sized here, before the first upload: a DBuf that grows inside decode() frees its old
  // block, and hipFree waits for the whole device -- ranges already in flight included.  A
  // context's first call, or one larger than any before it, still grows them on the way.
  if (c->wire_hint) {
    CHK(size_votes(std::min(U / 2 + 1, c->wire_hint + c->wire_hint / 4 + 4096)));
    for (size_t k = 0; k < R; ++k) {
      const uint64_t share = (uint64_t)((double)c->wire_hint * (double)(ub[k + 1] - ub[k]) / (double)std::max<uint64_t>(U, 1));
      CHK(c->rec_works[k]->ensure(
          hlc::recover_range_words(std::min((ub[k + 1] - ub[k]) / 2 + 1, share + share / 4 + 4096)) * 4));
    }
  }
  // 2. the wire bytes, range by range, piece by piece
  for (size_t k = 0; k < R; ++k) {
    for (uint64_t lo = ub[k]; lo < ub[k + 1];) {
      const uint64_t hi = std::min(ub[k + 1], lo + chunk);
      if (wire_pinned) {
        CHK(st.up_from(o[3] + lo, wire + lo, hi - lo));
      } else {
        pool.run([&](int t, int T) {
          const uint64_t d0 = lo + (hi - lo) * t / T, d1 = lo + (hi - lo) * (t + 1) / T;
          if (d1 > d0) stage_copy(st.P + o[3] + d0, wire + d0, d1 - d0, st.nt);
        });
        CHK(st.up(o[3] + lo, hi - lo));
      }
      lo = hi;
      CHK(drain_counts(false));
    }
    HIPCHK(hipEventRecord(c->ev_up[k], c->copy));
    tr.mark("staged_" + std::to_string(k));
    tr.ev("landed_" + std::to_string(k), c->copy);
    if (overflow) break;
    CHK(walk(k));
    ++walked;
    CHK(drain_counts(false));
  }
  CHK(drain_counts(true));
  if (overflow) {  // more votes than the first range's density promised: unpipelined, from the start
    tr.fact("overflow_capacity", (double)N);
    st.drain();
    guard.armed = false;
    c->wire_hint = std::max(c->wire_hint, N + 1);
    return wire_host_plain(c, wire, wire_len, moff, mlen, nm, scope, n_scope, now, out_res, out_wire, out_n_votes);
  }
  // 4. validation over every decoded vote, one finish after the ranges' main stages
  HIPCHK(hipEventRecord(c->ev_rest, c->dec));  // every range decoded, first-error passes included
  HIPCHK(hipStreamWaitEvent(s, c->ev_rest, 0));
  dv.n = base;
  CHK(validate_device(c, &dv, dprops, nm, now, c->w_res.as<hlc_result>(), nullptr, nullptr, nullptr, s, fronts.data(),
                      (int)fronts.size(), N));
  hlc::launch_wire_results(nm, dwout, c->w_res.as<hlc_result>(), s);
  HIPCHK(hipGetLastError());
  tr.ev("kernels_end", s);
  HIPCHK(hipMemcpyAsync(c->pin_out.p, c->w_res.p, nm * sizeof(hlc_result), hipMemcpyDeviceToHost, s));
  if (out_wire) HIPCHK(hipMemcpyAsync(c->pin_out.at(r1), dwout, nm * sizeof(hlc_wire_proposal), hipMemcpyDeviceToHost, s));
  HIPCHK(hipEventRecord(c->ev_done, s));
  tr.ev("outputs_landed", s);
  tr.mark("enqueued");
  HIPCHK(hipEventSynchronize(c->ev_done));
  guard.armed = false;
  tr.mark("device_done");
  std::memcpy(out_res, c->pin_out.p, nm * sizeof(hlc_result));
  if (out_wire) std::memcpy(out_wire, c->pin_out.at(r1), nm * sizeof(hlc_wire_proposal));
  if (out_n_votes) *out_n_votes = base;
  tr.fact("capacity", (double)N);
  c->wire_hint = std::max(c->wire_hint, base);
  tr.mark("outputs_copied");
  return 0;
}

}  // namespace

extern "C" {

const char* hlc_last_error(void) { return g_err.c_str(); }

int hlc_host_alloc(uint64_t bytes, void** out) {
  if (!out) return set_err(HLC_EINVAL, "out is NULL");
  *out = nullptr;
  if (!bytes) return 0;
  HIPCHK(hipHostMalloc(out, bytes, hipHostMallocDefault));
  return 0;
}

void hlc_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

int hlc_abi_version(void) { return HLC_ABI_VERSION; }

int hlc_host_threads(void) { return read_env().host_threads; }

const char* hlc_ctx_last_host_trace(hlc_ctx* ctx) {
  // a copy taken under the context's lock, valid on this thread until its next call
  thread_local std::string copy;
  if (!ctx) return "";
  std::lock_guard<std::mutex> lk(ctx->mu);
  copy = ctx->last_trace;
  return copy.c_str();
}

int hlc_ctx_set_option(hlc_ctx* ctx, int option, int64_t value) {
  if (!ctx) return set_err(HLC_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(ctx->mu);
  Options& o = ctx->opt;
  auto bad = [&]() { return set_err(HLC_EINVAL, "option " + std::to_string(option) + ": value " +
                                                    std::to_string(value) + " out of range"); };
  switch (option) {
    case HLC_OPT_HOST_THREADS:
      if (value < 1 || value > 64) return bad();
      o.host_threads = (int)value;
      break;
    case HLC_OPT_POOL_BIND:
      if (value < 0 || value > 2) return bad();
      o.pool_bind = (int)value;
      break;
    case HLC_OPT_NT_COPY: o.nt_copy = value != 0; break;
    case HLC_OPT_SPLIT_VOTES:
      if (value < -1) return bad();
      if (value == -1) o.split_votes = Options().split_votes;  // the library default
      else o.split_votes.assign(1, (uint64_t)value);
      break;
    case HLC_OPT_HOST_TRACE:
      if (value < 0 || value > 2) return bad();
      o.host_trace = (int)value;
      break;
    case HLC_OPT_FIRST_BATCH:
      if (value < 0 || value > 64) return bad();
      o.first_batch = (int)value;
      break;
    case HLC_OPT_REST_PIECES:
      if (value < 1 || value > 64) return bad();
      o.rest_pieces = (int)value;
      break;
    case HLC_OPT_WIRE_SPLIT_BYTES:
      if (value < -1) return bad();
      if (value == -1) o.wire_split_bytes = Options().wire_split_bytes;  // the library default
      else o.wire_split_bytes.assign(1, (uint64_t)value);
      break;
    case HLC_OPT_WIRE_FRONT_CAP:
      if (value < 0) return bad();
      o.wire_front_cap = (uint64_t)value;
      break;
    case HLC_OPT_SPLIT_VOTES_APPEND:
      if (value < 0 || o.split_votes.size() >= 16) return bad();
      o.split_votes.push_back((uint64_t)value);
      break;
    case HLC_OPT_WIRE_SPLIT_BYTES_APPEND:
      if (value < 0 || o.wire_split_bytes.size() >= 16) return bad();
      o.wire_split_bytes.push_back((uint64_t)value);
      break;
    case HLC_OPT_WIRE_CHUNK:
      if (value < 1) return bad();
      o.wire_chunk = std::max<uint64_t>((uint64_t)value, 4096);  // (as the environment's value: at least 4 KiB)
      break;
    case HLC_OPT_REC_FORCE_EXACT: o.rec_force_exact = value != 0; break;
    case HLC_OPT_SERIAL_STAGES: o.serial_stages = value != 0; break;
    case HLC_OPT_WIRE_PIPELINE: o.wire_pipeline = value != 0; break;
    case HLC_OPT_WIRE_WALK:
      if (value < -1 || value > 1) return bad();
      o.wire_walk = (int)value;
      break;
    case HLC_OPT_EARLY_COMB:
      if (value < 0 || value > 3) return bad();
      o.early_comb = (int)value;
      break;
    default: return set_err(HLC_EINVAL, "unknown option " + std::to_string(option));
  }
  return 0;
}

int hlc_ctx_get_option(hlc_ctx* ctx, int option, int64_t* value) {
  if (!ctx || !value) return set_err(HLC_EINVAL, "NULL argument");
  std::lock_guard<std::mutex> lk(ctx->mu);
  const Options& o = ctx->opt;
  switch (option) {
    case HLC_OPT_HOST_THREADS: *value = o.host_threads; break;
    case HLC_OPT_POOL_BIND: *value = o.pool_bind; break;
    case HLC_OPT_NT_COPY: *value = o.nt_copy; break;
    case HLC_OPT_SPLIT_VOTES: *value = o.split_votes.empty() ? 0 : (int64_t)o.split_votes[0]; break;
    case HLC_OPT_HOST_TRACE: *value = o.host_trace; break;
    case HLC_OPT_FIRST_BATCH: *value = o.first_batch; break;
    case HLC_OPT_REST_PIECES: *value = o.rest_pieces; break;
    case HLC_OPT_WIRE_SPLIT_BYTES: *value = o.wire_split_bytes.empty() ? 0 : (int64_t)o.wire_split_bytes[0]; break;
    case HLC_OPT_WIRE_FRONT_CAP: *value = (int64_t)o.wire_front_cap; break;
    case HLC_OPT_WIRE_CHUNK: *value = (int64_t)o.wire_chunk; break;
    case HLC_OPT_REC_FORCE_EXACT: *value = o.rec_force_exact; break;
    case HLC_OPT_SERIAL_STAGES: *value = o.serial_stages; break;
    case HLC_OPT_WIRE_PIPELINE: *value = o.wire_pipeline; break;
    case HLC_OPT_WIRE_WALK: *value = o.wire_walk; break;
    case HLC_OPT_EARLY_COMB: *value = o.early_comb; break;
    default: return set_err(HLC_EINVAL, "unknown option " + std::to_string(option));
  }
  return 0;
}

int hlc_ctx_create(int device, hlc_ctx** out) {
  if (!out) return set_err(HLC_EINVAL, "out is NULL");
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= device || device < 0)
    return set_err(HLC_ENODEV, "no HIP device with that ordinal");
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return set_err(HLC_ENODEV, std::string("libhlc is built for gfx950, device is ") + prop.gcnArchName);
  hlc_ctx* c = new hlc_ctx();
  c->device = device;
  c->opt = read_env();  // the options' defaults: the environment, read here only
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      create_aux(c) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_prep, hipEventDisableTiming) != hipSuccess) {
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    delete c;
    return set_err(HLC_EDEVICE, "stream creation failed");
  }
  // the fixed-base tables: built by the first context on this device, shared by the others (gen_tables)
  if (const int rc = gen_tables(device, c->stream, c->gen)) {
    hipStream_t st = c->stream, ax = c->aux;
    delete c;
    (void)hipStreamDestroy(st);
    (void)hipStreamDestroy(ax);
    return rc;
  }
  c->gtab = reinterpret_cast<const uint32_t*>(c->gen->g);
  c->fbtab = reinterpret_cast<const uint32_t*>(c->gen->fb);
  *out = c;
  return 0;
}

void hlc_ctx_destroy(hlc_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  destroy_ctx(ctx);
}

int hlc_ctx_reserve(hlc_ctx* ctx, uint64_t max_votes, uint64_t max_proposals, uint64_t max_bytes) {
  if (!ctx) return set_err(HLC_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  const uint64_t n = max_votes;
  CHK(reserve_validate(ctx, n, max_proposals));
  for (DBuf* b : {&ctx->sha_sz, &ctx->sha_off, &ctx->kec_sz, &ctx->kec_off}) CHK(b->ensure(n * 8));
  CHK(ctx->sha_dig.ensure(n * 32));
  CHK(ctx->sha_buf.ensure(n * 128 + max_bytes + 64));
  CHK(ctx->kec_buf.ensure(n * 272 + max_bytes + 136));
  return 0;
}

int hlc_ctx_set_kernel_timing(hlc_ctx* ctx, int enable) {
  if (!ctx) return set_err(HLC_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->timing = enable == HLC_TIMING_RECOVERY ? HLC_TIMING_RECOVERY : (enable ? HLC_TIMING_ALL : 0);
  return 0;
}

int hlc_ctx_set_clock_probe(hlc_ctx* ctx, int enable) {
  if (!ctx) return set_err(HLC_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->clock_probe = enable != 0;
  ctx->clk_waves = 0;
  return 0;
}

int hlc_ctx_clock_probe(hlc_ctx* ctx, double* median_ghz, double* min_ghz, double* max_ghz, uint64_t* waves) {
  if (!ctx) return set_err(HLC_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  std::vector<double> ghz;
  if (ctx->clk_waves && ctx->clk_buf.p) {
    HIPCHK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(4 * ctx->clk_waves);
    HIPCHK(hipMemcpy(h.data(), ctx->clk_buf.p, h.size() * 8, hipMemcpyDeviceToHost));
    for (uint64_t w = 0; w < ctx->clk_waves; ++w) {  // (start core, start ref, end core, end ref) per wave
      const unsigned long long* t = &h[4 * w];
      if (t[2] > t[0] && t[3] > t[1]) ghz.push_back(0.1 * (double)(t[2] - t[0]) / (double)(t[3] - t[1]));
    }
  }
  if (ghz.empty()) return set_err(HLC_EINVAL, "no k_rec_main launch stamped since hlc_ctx_set_clock_probe(ctx, 1)");
  std::sort(ghz.begin(), ghz.end());
  if (median_ghz) *median_ghz = ghz[ghz.size() / 2];
  if (min_ghz) *min_ghz = ghz.front();
  if (max_ghz) *max_ghz = ghz.back();
  if (waves) *waves = ghz.size();
  return 0;
}

int hlc_ctx_take_kernel_time(hlc_ctx* ctx, double* recover_ms, uint64_t* recover_launches, double* call_ms,
                             uint64_t* calls) {
  if (!ctx) return set_err(HLC_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  double rsum = 0, csum = 0;
  for (auto* vec : {&ctx->rec_ev, &ctx->rec_prep_ev, &ctx->call_ev}) {
    for (auto& pr : *vec) {
      HIPCHK(hipEventSynchronize(pr.second));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, pr.first, pr.second));
      (vec == &ctx->call_ev ? csum : rsum) += ms;
    }
  }
  if (recover_ms) *recover_ms = rsum;
  if (recover_launches) *recover_launches = ctx->rec_ev.size();
  if (call_ms) *call_ms = csum;
  if (calls) *calls = ctx->call_ev.size();
  for (auto* vec : {&ctx->rec_ev, &ctx->rec_prep_ev, &ctx->call_ev}) {
    for (auto& pr : *vec) {
      ctx->ev_pool.push_back(pr.first);
      if (vec != &ctx->call_ev) ctx->ev_pool.push_back(pr.second);  // (a call's end is chain_ev's)
    }
    vec->clear();
  }
  return 0;
}

int hlc_ctx_take_chain_time(hlc_ctx* ctx, double* chain_ms, uint64_t* launches) {
  if (!ctx) return set_err(HLC_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  double sum = 0;
  for (auto* vec : {&ctx->chain_ev, &ctx->chain_aux_ev}) {
    for (auto& pr : *vec) {
      HIPCHK(hipEventSynchronize(pr.second));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, pr.first, pr.second));
      sum += ms;
    }
  }
  if (chain_ms) *chain_ms = sum;
  if (launches) *launches = ctx->chain_ev.size();
  for (auto& pr : ctx->chain_aux_ev) {
    ctx->ev_pool.push_back(pr.first);
    ctx->ev_pool.push_back(pr.second);
  }
  ctx->chain_aux_ev.clear();
  for (auto& pr : ctx->chain_ev) {
    ctx->ev_pool.push_back(pr.first);
    ctx->ev_pool.push_back(pr.second);
  }
  ctx->chain_ev.clear();
  return 0;
}

int hlc_validate_proposals_device(hlc_ctx* ctx, const hlc_votes* votes, const hlc_proposal* proposals,
                                  uint64_t n_proposals, uint64_t now, hlc_result* out_results,
                                  uint8_t* out_vote_status, uint8_t* out_vote_reason, uint8_t* out_recovered,
                                  void* stream) {
  if (!ctx || !votes || (n_proposals && (!proposals || !out_results)))
    return set_err(HLC_EINVAL, "NULL argument");
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
  return validate_device(ctx, votes, proposals, n_proposals, now, out_results, out_vote_status, out_vote_reason,
                         out_recovered, s);
}

int hlc_outcome_counts_device(hlc_ctx* ctx, const uint8_t* vote_status, uint64_t n_votes,
                              const hlc_result* results, uint64_t n_proposals, uint64_t* out_counts,
                              void* stream) {
  if (!ctx || !out_counts || (n_votes && !vote_status) || (n_proposals && !results))
    return set_err(HLC_EINVAL, "NULL argument");
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
  HIPCHK(hipMemsetAsync(out_counts, 0, 64 * sizeof(uint64_t), s));
  hlc::launch_outcome_hist(vote_status, n_votes, results, n_proposals,
                           reinterpret_cast<unsigned long long*>(out_counts), s);
  HIPCHK(hipGetLastError());
  return 0;
}

int hlc_validate_proposals(hlc_ctx* ctx, const hlc_votes* votes, const hlc_proposal* proposals,
                           uint64_t n_proposals, uint64_t now, hlc_result* out_results, uint8_t* out_vote_status,
                           uint8_t* out_vote_reason, uint8_t* out_recovered) {
  if (!ctx) return set_err(HLC_EINVAL, "ctx is NULL");
  if (!votes) return set_err(HLC_EINVAL, "votes is NULL");
  if (votes->n && (!votes->vote_id || !votes->proposal_id || !votes->timestamp || !votes->vote ||
                   !votes->field_off || !votes->field_len))
    return set_err(HLC_EINVAL, "NULL vote array");
  if (n_proposals && (!proposals || !out_results)) return set_err(HLC_EINVAL, "NULL proposals/results");
  for (uint64_t p = 0; p < n_proposals; ++p) {
    if (proposals[p].vote_begin + proposals[p].vote_count > votes->n ||
        proposals[p].vote_begin + proposals[p].vote_count < proposals[p].vote_begin)
      return set_err(HLC_EINVAL, "proposal vote range outside the vote batch");
  }
  if (votes->n > 0xFFFFFFF0ull) return set_err(HLC_EINVAL, "too many votes in one call (max 2^32-16)");
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  return validate_host(ctx, votes, proposals, n_proposals, now, out_results, out_vote_status, out_vote_reason,
                       out_recovered);
}

int hlc_decode_proposals(hlc_ctx* ctx, const uint8_t* wire, uint64_t wire_len, const uint64_t* msg_off,
                         const uint32_t* msg_len, uint64_t n_msgs, const hlc_scope_config* scope, uint64_t n_scope,
                         hlc_proposal* out_props, hlc_wire_proposal* out_wire, uint64_t* inout_n_votes,
                         uint32_t* vote_id, uint32_t* proposal_id, uint64_t* timestamp, uint8_t* vote,
                         uint64_t* field_off, uint32_t* field_len) {
  if (!ctx || !inout_n_votes || (n_msgs && !out_props)) return set_err(HLC_EINVAL, "NULL argument");
  CHK(check_wire_host(wire, wire_len, msg_off, msg_len, n_msgs, scope, n_scope));
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = ctx->stream;
  CHK(stage_wire(ctx, wire, wire_len, msg_off, msg_len, n_msgs, scope, n_scope, s));
  hlc_votes dv;
  uint64_t nv = 0;
  CHK(decode_device(ctx, ctx->w_wire.as<uint8_t>(), wire_len, ctx->w_moff.as<uint64_t>(), ctx->w_mlen.as<uint32_t>(),
                    n_msgs, ctx->w_scope.as<hlc_scope_config>(), n_scope, ctx->w_props.as<hlc_proposal>(),
                    ctx->w_wout.as<hlc_wire_proposal>(), &dv, &nv, s));
  if (n_msgs) {
    HIPCHK(hipMemcpyAsync(out_props, ctx->w_props.p, n_msgs * sizeof(hlc_proposal), hipMemcpyDeviceToHost, s));
    if (out_wire)
      HIPCHK(hipMemcpyAsync(out_wire, ctx->w_wout.p, n_msgs * sizeof(hlc_wire_proposal), hipMemcpyDeviceToHost, s));
  }
  const uint64_t cap = *inout_n_votes;
  *inout_n_votes = nv;
  const bool want = vote_id || proposal_id || timestamp || vote || field_off || field_len;
  int rc = 0;
  if (want && nv > cap) {
    rc = set_err(HLC_ERANGE, "vote capacity too small: " + std::to_string(nv) + " votes decoded");
  } else if (want && nv) {
    if (!vote_id || !proposal_id || !timestamp || !vote || !field_off || !field_len)
      return set_err(HLC_EINVAL, "vote output arrays must be all set or all NULL");
    HIPCHK(hipMemcpyAsync(vote_id, dv.vote_id, nv * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(proposal_id, dv.proposal_id, nv * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(timestamp, dv.timestamp, nv * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(vote, dv.vote, nv, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(field_off, dv.field_off, nv * 8 * HLC_NFIELDS, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(field_len, dv.field_len, nv * 4 * HLC_NFIELDS, hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  return rc;
}

int hlc_validate_wire_proposals_device(hlc_ctx* ctx, const uint8_t* wire, uint64_t wire_len, const uint64_t* msg_off,
                                       const uint32_t* msg_len, uint64_t n_msgs, const hlc_scope_config* scope,
                                       uint64_t n_scope, uint64_t now, hlc_result* out_results,
                                       hlc_wire_proposal* out_wire, void* stream) {
  if (!ctx || (n_msgs && (!msg_off || !msg_len || !scope || !out_results)))
    return set_err(HLC_EINVAL, "NULL argument");
  if (n_msgs && n_scope != 1 && n_scope != n_msgs) return set_err(HLC_EINVAL, "n_scope must be 1 or n_msgs");
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
  CHK(ctx->w_props.ensure(n_msgs * sizeof(hlc_proposal) + 16));
  hlc_wire_proposal* wout = out_wire;
  if (!wout) {
    CHK(ctx->w_wout.ensure(n_msgs * sizeof(hlc_wire_proposal) + 16));
    wout = ctx->w_wout.as<hlc_wire_proposal>();
  }
  hlc_votes dv;
  uint64_t nv = 0;
  CHK(decode_device(ctx, wire, wire_len, msg_off, msg_len, n_msgs, scope, n_scope, ctx->w_props.as<hlc_proposal>(),
                    wout, &dv, &nv, s));
  CHK(validate_device(ctx, &dv, ctx->w_props.as<hlc_proposal>(), n_msgs, now, out_results, nullptr, nullptr, nullptr,
                      s));
  hlc::launch_wire_results(n_msgs, wout, out_results, s);
  HIPCHK(hipGetLastError());
  return 0;
}

int hlc_validate_wire_proposals(hlc_ctx* ctx, const uint8_t* wire, uint64_t wire_len, const uint64_t* msg_off,
                                const uint32_t* msg_len, uint64_t n_msgs, const hlc_scope_config* scope,
                                uint64_t n_scope, uint64_t now, hlc_result* out_results, hlc_wire_proposal* out_wire,
                                uint64_t* out_n_votes) {
  if (!ctx || (n_msgs && !out_results)) return set_err(HLC_EINVAL, "NULL argument");
  CHK(check_wire_host(wire, wire_len, msg_off, msg_len, n_msgs, scope, n_scope));
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  if (!ctx->opt.wire_pipeline)  // A/B arm: unpipelined
    return wire_host_plain(ctx, wire, wire_len, msg_off, msg_len, n_msgs, scope, n_scope, now, out_results, out_wire,
                           out_n_votes);
  return validate_wire_host(ctx, wire, wire_len, msg_off, msg_len, n_msgs, scope, n_scope, now, out_results, out_wire,
                            out_n_votes);
}

}  // extern "C"

namespace {

// process_incoming_vote over device-resident inputs (see hlc_process_votes); outputs on device.
// (owner_off != nullptr: owners is an arena of any-length identities; verdicts != nullptr: the scheme step
// is the caller's, hlc_process_votes_verdicts)
int process_votes_device(hlc_ctx* ctx, const hlc_votes* dv, const uint32_t* vsess, hlc_session* dss,
                         uint64_t n_sessions, const uint8_t* owners, const uint32_t* owner_session, uint64_t n_owners,
                         uint64_t now, uint8_t* st, uint8_t* tr, uint8_t* ins, uint8_t* reason, hipStream_t s,
                         const uint64_t* owner_off = nullptr, const uint32_t* owner_len = nullptr,
                         const uint8_t* verdicts = nullptr) {
  const uint64_t n = dv->n;
  CHK(ctx->s_props.ensure(n_sessions * sizeof(hlc_proposal) + 16));
  hlc_proposal* dprops = ctx->s_props.as<hlc_proposal>();
  hlc::launch_sessions_to_props(dss, n_sessions, dprops, s);
  // 1. validate_vote for every vote against its session's proposal (same kernels as validate-many)
  CHK(ctx->status.ensure(n + 1));
  uint8_t* rs = reason;
  if (!rs) {
    CHK(ctx->reason.ensure(n + 1));
    rs = ctx->reason.as<uint8_t>();
  }
  CHK(ctx->flag.ensure(16));
  HIPCHK(hipMemsetAsync(ctx->flag.p, 0, sizeof(uint32_t), s));
  if (n)
    CHK(vote_stage(ctx, dv, vsess, dprops, n_sessions, now, ctx->status.as<uint8_t>(), rs, nullptr, nullptr, nullptr, s,
                   nullptr, 0, 0, verdicts));
  // 2. each session's votes in delivery order
  CHK(ctx->s_keys.ensure(n * 4 + 4));
  CHK(ctx->s_iota.ensure(n * 4 + 4));
  CHK(ctx->s_order.ensure(n * 4 + 4));
  size_t tb = 0;
  HIPCHK(hlc::launch_sort_by_session(vsess, n, ctx->s_keys.as<uint32_t>(), ctx->s_iota.as<uint32_t>(),
                              ctx->s_order.as<uint32_t>(), nullptr, tb, s));
  CHK(ctx->s_sort_tmp.ensure(tb + 16));
  HIPCHK(hlc::launch_sort_by_session(vsess, n, ctx->s_keys.as<uint32_t>(), ctx->s_iota.as<uint32_t>(),
                              ctx->s_order.as<uint32_t>(), ctx->s_sort_tmp.p, tb, s));
  CHK(ctx->s_segb.ensure(n_sessions * 4 + 4));
  CHK(ctx->s_sege.ensure(n_sessions * 4 + 4));
  HIPCHK(hipMemsetAsync(ctx->s_segb.p, 0, n_sessions * 4 + 4, s));
  HIPCHK(hipMemsetAsync(ctx->s_sege.p, 0, n_sessions * 4 + 4, s));
  hlc::launch_segments(ctx->s_keys.as<uint32_t>(), n, ctx->s_segb.as<uint32_t>(), ctx->s_sege.as<uint32_t>(), s);
  // 3. (session, owner) table: existing owner maps, then add_vote in order per session
  uint64_t cap = 64;
  while (cap < 2 * (n + n_owners)) cap <<= 1;
  CHK(ctx->s_tab.ensure(cap * 8));  // keys, then the minimum delivery position per key
  HIPCHK(hipMemsetAsync(ctx->s_tab.p, 0xFF, cap * 8, s));
  CHK(ctx->s_slot.ensure(n * 4 + 4));
  CHK(ctx->s_dup.ensure(n + 1));
  hlc::launch_stream_init(n, vsess, ctx->status.as<uint8_t>(), st, tr, ins, s);
  uint32_t* tab = ctx->s_tab.as<uint32_t>();
  hlc::launch_dup_flags(tab, tab + cap, (uint32_t)(cap - 1), owners, owner_session, n_owners, dv, vsess, st,
                        ctx->s_slot.as<uint32_t>(), ctx->s_dup.as<uint8_t>(), s, owner_off, owner_len);
  hlc::launch_apply_votes(dss, n_sessions, ctx->s_segb.as<uint32_t>(), ctx->s_sege.as<uint32_t>(),
                          ctx->s_order.as<uint32_t>(), dv, now, ctx->s_dup.as<uint8_t>(), st, tr, ins, s);
  HIPCHK(hipGetLastError());
  return 0;
}

}  // namespace

extern "C" {

int hlc_process_votes_device(hlc_ctx* ctx, const hlc_votes* votes, const uint32_t* vote_session,
                             hlc_session* sessions, uint64_t n_sessions, const uint8_t* owners,
                             const uint32_t* owner_session, uint64_t n_owners, uint64_t now, uint8_t* out_status,
                             uint8_t* out_transition, uint8_t* out_inserted, uint8_t* out_reason, void* stream) {
  if (!ctx || !votes) return set_err(HLC_EINVAL, "NULL argument");
  if (votes->n && (!vote_session || !out_status || !out_transition || !out_inserted))
    return set_err(HLC_EINVAL, "NULL vote_session / output array");
  if (n_sessions >= hlc::NO_PROP || votes->n + n_owners > 0xFFFFFFF0ull) return set_err(HLC_EINVAL, "batch too large");
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
  return process_votes_device(ctx, votes, vote_session, sessions, n_sessions, owners, owner_session, n_owners, now,
                              out_status, out_transition, out_inserted, out_reason, s);
}

int hlc_process_votes(hlc_ctx* ctx, const hlc_votes* votes, const uint32_t* vote_session, hlc_session* sessions,
                      uint64_t n_sessions, const uint8_t* owners, const uint32_t* owner_session, uint64_t n_owners,
                      uint64_t now, uint8_t* out_status, uint8_t* out_transition, uint8_t* out_inserted,
                      uint8_t* out_reason) {
  if (!ctx) return set_err(HLC_EINVAL, "ctx is NULL");
  CHK(check_votes_host(votes));
  const uint64_t n = votes->n;
  if (n && (!vote_session || !out_status || !out_transition || !out_inserted))
    return set_err(HLC_EINVAL, "NULL vote_session / output array");
  if (n_sessions && !sessions) return set_err(HLC_EINVAL, "sessions is NULL");
  if (n_owners && (!owners || !owner_session)) return set_err(HLC_EINVAL, "NULL owner arrays");
  if (n_sessions >= hlc::NO_PROP || n + n_owners > 0xFFFFFFF0ull) return set_err(HLC_EINVAL, "batch too large");
  for (uint64_t i = 0; i < n; ++i)
    if (vote_session[i] != hlc::NO_PROP && vote_session[i] >= n_sessions)
      return set_err(HLC_EINVAL, "vote_session index out of range");
  for (uint64_t k = 0; k < n_owners; ++k)
    if (owner_session[k] >= n_sessions) return set_err(HLC_EINVAL, "owner_session index out of range");
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = ctx->stream;
  hlc_votes dv;
  CHK(stage_votes(ctx, votes, &dv, s));
  CHK(upload(ctx->s_vsess, vote_session, n, s));
  CHK(upload(ctx->s_sessions, sessions, n_sessions, s));
  CHK(upload(ctx->s_owners, owners, n_owners * 20, s));
  CHK(upload(ctx->s_osess, owner_session, n_owners, s));
  CHK(ctx->s_st.ensure(n + 1));
  CHK(ctx->s_tr.ensure(n + 1));
  CHK(ctx->s_ins.ensure(n + 1));
  CHK(ctx->reason.ensure(n + 1));
  hlc_session* dss = ctx->s_sessions.as<hlc_session>();
  CHK(process_votes_device(ctx, &dv, ctx->s_vsess.as<uint32_t>(), dss, n_sessions, ctx->s_owners.as<uint8_t>(),
                           ctx->s_osess.as<uint32_t>(), n_owners, now, ctx->s_st.as<uint8_t>(), ctx->s_tr.as<uint8_t>(),
                           ctx->s_ins.as<uint8_t>(), ctx->reason.as<uint8_t>(), s));
  if (n) {
    HIPCHK(hipMemcpyAsync(out_status, ctx->s_st.p, n, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out_transition, ctx->s_tr.p, n, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out_inserted, ctx->s_ins.p, n, hipMemcpyDeviceToHost, s));
    if (out_reason) HIPCHK(hipMemcpyAsync(out_reason, ctx->reason.p, n, hipMemcpyDeviceToHost, s));
  }
  if (n_sessions)
    HIPCHK(hipMemcpyAsync(sessions, dss, n_sessions * sizeof(hlc_session), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}

int hlc_process_votes_verdicts(hlc_ctx* ctx, const hlc_votes* votes, const uint32_t* vote_session,
                               hlc_session* sessions, uint64_t n_sessions, const uint8_t* owner_bytes,
                               uint64_t owner_bytes_len, const uint64_t* owner_off, const uint32_t* owner_len,
                               const uint32_t* owner_session, uint64_t n_owners, uint64_t now, const uint8_t* verdicts,
                               uint8_t* out_status, uint8_t* out_transition, uint8_t* out_inserted,
                               uint8_t* out_reason) {
  if (!ctx) return set_err(HLC_EINVAL, "ctx is NULL");
  CHK(check_votes_host(votes));
  const uint64_t n = votes->n;
  if (n && (!vote_session || !out_status || !out_transition || !out_inserted || !verdicts))
    return set_err(HLC_EINVAL, "NULL vote_session / verdicts / output array");
  if (n_sessions && !sessions) return set_err(HLC_EINVAL, "sessions is NULL");
  if (n_owners && (!owner_off || !owner_len || !owner_session)) return set_err(HLC_EINVAL, "NULL owner arrays");
  if (n_sessions >= hlc::NO_PROP || n + n_owners > 0xFFFFFFF0ull) return set_err(HLC_EINVAL, "batch too large");
  CHK(check_verdicts(verdicts, n));
  for (uint64_t i = 0; i < n; ++i)
    if (vote_session[i] != hlc::NO_PROP && vote_session[i] >= n_sessions)
      return set_err(HLC_EINVAL, "vote_session index out of range");
  for (uint64_t k = 0; k < n_owners; ++k) {
    if (owner_session[k] >= n_sessions) return set_err(HLC_EINVAL, "owner_session index out of range");
    if (owner_len[k] && (!owner_bytes || owner_off[k] + owner_len[k] > owner_bytes_len ||
                         owner_off[k] + owner_len[k] < owner_off[k]))
      return set_err(HLC_EINVAL, "owner (offset, length) outside owner_bytes");
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = ctx->stream;
  hlc_votes dv;
  CHK(stage_votes(ctx, votes, &dv, s));
  CHK(upload(ctx->s_vsess, vote_session, n, s));
  CHK(upload(ctx->s_sessions, sessions, n_sessions, s));
  CHK(upload(ctx->s_owners, owner_bytes, owner_bytes ? owner_bytes_len : 0, s));
  CHK(upload(ctx->in_off3, owner_off, n_owners, s));
  CHK(upload(ctx->in_len3, owner_len, n_owners, s));
  CHK(upload(ctx->s_osess, owner_session, n_owners, s));
  CHK(upload(ctx->in_verdict, verdicts, n, s));
  CHK(ctx->s_st.ensure(n + 1));
  CHK(ctx->s_tr.ensure(n + 1));
  CHK(ctx->s_ins.ensure(n + 1));
  CHK(ctx->reason.ensure(n + 1));
  hlc_session* dss = ctx->s_sessions.as<hlc_session>();
  CHK(process_votes_device(ctx, &dv, ctx->s_vsess.as<uint32_t>(), dss, n_sessions, ctx->s_owners.as<uint8_t>(),
                           ctx->s_osess.as<uint32_t>(), n_owners, now, ctx->s_st.as<uint8_t>(), ctx->s_tr.as<uint8_t>(),
                           ctx->s_ins.as<uint8_t>(), ctx->reason.as<uint8_t>(), s, ctx->in_off3.as<uint64_t>(),
                           ctx->in_len3.as<uint32_t>(), ctx->in_verdict.as<uint8_t>()));
  if (n) {
    HIPCHK(hipMemcpyAsync(out_status, ctx->s_st.p, n, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out_transition, ctx->s_tr.p, n, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out_inserted, ctx->s_ins.p, n, hipMemcpyDeviceToHost, s));
    if (out_reason) HIPCHK(hipMemcpyAsync(out_reason, ctx->reason.p, n, hipMemcpyDeviceToHost, s));
  }
  if (n_sessions)
    HIPCHK(hipMemcpyAsync(sessions, dss, n_sessions * sizeof(hlc_session), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}

int hlc_validate_proposals_verdicts_device(hlc_ctx* ctx, const hlc_votes* votes, const hlc_proposal* proposals,
                                           uint64_t n_proposals, uint64_t now, const uint8_t* verdicts,
                                           hlc_result* out_results, uint8_t* out_vote_status,
                                           uint8_t* out_vote_reason, void* stream) {
  if (!ctx || !votes || (votes->n && !verdicts) || (n_proposals && (!proposals || !out_results)))
    return set_err(HLC_EINVAL, "NULL argument");
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
  return validate_device(ctx, votes, proposals, n_proposals, now, out_results, out_vote_status, out_vote_reason,
                         nullptr, s, nullptr, 0, 0, verdicts);
}

int hlc_validate_proposals_verdicts(hlc_ctx* ctx, const hlc_votes* votes, const hlc_proposal* proposals,
                                    uint64_t n_proposals, uint64_t now, const uint8_t* verdicts,
                                    hlc_result* out_results, uint8_t* out_vote_status, uint8_t* out_vote_reason) {
  if (!ctx) return set_err(HLC_EINVAL, "ctx is NULL");
  CHK(check_votes_host(votes));
  const uint64_t n = votes->n;
  if (n && !verdicts) return set_err(HLC_EINVAL, "verdicts is NULL");
  if (n_proposals && (!proposals || !out_results)) return set_err(HLC_EINVAL, "NULL proposals/results");
  for (uint64_t p = 0; p < n_proposals; ++p) {
    if (proposals[p].vote_begin + proposals[p].vote_count > n ||
        proposals[p].vote_begin + proposals[p].vote_count < proposals[p].vote_begin)
      return set_err(HLC_EINVAL, "proposal vote range outside the vote batch");
  }
  if (n > 0xFFFFFFF0ull) return set_err(HLC_EINVAL, "too many votes in one call (max 2^32-16)");
  CHK(check_verdicts(verdicts, n));
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = ctx->stream;
  hlc_votes dv;
  CHK(stage_votes(ctx, votes, &dv, s));
  CHK(upload(ctx->in_props, proposals, n_proposals, s));
  CHK(upload(ctx->in_verdict, verdicts, n, s));
  CHK(ctx->out_res.ensure(n_proposals * sizeof(hlc_result) + 16));
  CHK(ctx->out_status.ensure(n + 1));
  CHK(ctx->out_reason.ensure(n + 1));
  CHK(validate_device(ctx, &dv, ctx->in_props.as<hlc_proposal>(), n_proposals, now, ctx->out_res.as<hlc_result>(),
                      ctx->out_status.as<uint8_t>(), ctx->out_reason.as<uint8_t>(), nullptr, s, nullptr, 0, 0,
                      ctx->in_verdict.as<uint8_t>()));
  if (n_proposals)
    HIPCHK(hipMemcpyAsync(out_results, ctx->out_res.p, n_proposals * sizeof(hlc_result), hipMemcpyDeviceToHost, s));
  if (n && out_vote_status) HIPCHK(hipMemcpyAsync(out_vote_status, ctx->out_status.p, n, hipMemcpyDeviceToHost, s));
  if (n && out_vote_reason) HIPCHK(hipMemcpyAsync(out_vote_reason, ctx->out_reason.p, n, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}

int hlc_encode_vote_payloads(hlc_ctx* ctx, const hlc_votes* votes, uint64_t* out_off, uint32_t* out_len,
                             uint8_t* out_bytes, uint64_t cap, uint64_t* out_total) {
  if (!ctx || !out_total) return set_err(HLC_EINVAL, "NULL argument");
  CHK(check_votes_host(votes));
  const uint64_t n = votes->n;
  if (n && (!out_off || !out_len)) return set_err(HLC_EINVAL, "NULL out_off / out_len");
  if (n > 0x7FFFFFF0ull) return set_err(HLC_EINVAL, "too many votes in one call (max 2^31-16)");
  *out_total = 0;
  if (!n) return 0;
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = ctx->stream;
  hlc_votes dv;
  CHK(stage_votes(ctx, votes, &dv, s));
  CHK(ctx->kec_sz.ensure(n * 8));
  CHK(ctx->kec_off.ensure(n * 8));
  CHK(ctx->out_misc.ensure(n * 4 + 16));
  hlc::launch_payload_sizes(&dv, n, ctx->kec_sz.as<uint64_t>(), ctx->out_misc.as<uint32_t>(), s);
  HIPCHK(hipGetLastError());
  uint64_t total = 0;
  CHK(scan_sizes(ctx, n, ctx->kec_sz.as<uint64_t>(), ctx->kec_off.as<uint64_t>(), &total, s));  // (synchronises)
  *out_total = total;
  HIPCHK(hipMemcpyAsync(out_off, ctx->kec_off.p, n * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(out_len, ctx->out_misc.p, n * 4, hipMemcpyDeviceToHost, s));
  int rc = 0;
  if (out_bytes && total > cap) {
    rc = set_err(HLC_ERANGE, "payload capacity too small: " + std::to_string(total) + " bytes needed");
  } else if (out_bytes && total) {
    CHK(ctx->kec_buf.ensure(total + 16));
    hlc::launch_encode_payloads(&dv, n, ctx->kec_off.as<uint64_t>(), ctx->kec_buf.as<uint8_t>(), s);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out_bytes, ctx->kec_buf.p, total, hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  return rc;
}

int hlc_compute_vote_hashes(hlc_ctx* ctx, const hlc_votes* votes, uint8_t* out_hash32) {
  if (!ctx || !out_hash32) return set_err(HLC_EINVAL, "NULL argument");
  CHK(check_votes_host(votes));
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = ctx->stream;
  const uint64_t n = votes->n;
  if (!n) return 0;
  hlc_votes dv;
  CHK(stage_votes(ctx, votes, &dv, s));
  CHK(run_prehash(ctx, &dv, n, hlc::MSG_VOTE, nullptr, nullptr, nullptr, s));
  HIPCHK(hipMemcpyAsync(out_hash32, ctx->sha_dig.p, n * 32, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}

int hlc_eth_verify_batch(hlc_ctx* ctx, uint64_t n, const uint8_t* bytes, uint64_t bytes_len, const uint64_t* id_off,
                         const uint32_t* id_len, const uint64_t* payload_off, const uint32_t* payload_len,
                         const uint64_t* sig_off, const uint32_t* sig_len, uint8_t* out_status, uint8_t* out_addr) {
  if (!ctx || (n && (!id_off || !id_len || !payload_off || !payload_len || !sig_off || !sig_len || !out_status)))
    return set_err(HLC_EINVAL, "NULL argument");
  if (!n) return 0;
  if (n > 0xFFFFFFF0ull) return set_err(HLC_EINVAL, "too many items in one call (max 2^32-16)");
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  return verify_host(ctx, n, bytes, bytes_len, id_off, id_len, payload_off, payload_len, sig_off, sig_len, out_status,
                     out_addr);
}

int hlc_consensus_timeout_batch(hlc_ctx* ctx, uint64_t n, const hlc_session_tally* sessions, uint8_t* out_state,
                                uint8_t* out_status) {
  if (!ctx || (n && (!sessions || !out_state || !out_status))) return set_err(HLC_EINVAL, "NULL argument");
  if (!n) return 0;
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = ctx->stream;
  CHK(upload(ctx->in_props, sessions, n, s));
  CHK(ctx->out_misc.ensure(2 * n + 16));
  uint8_t* d_state = ctx->out_misc.as<uint8_t>();
  uint8_t* d_status = d_state + n;
  hlc::launch_timeout(n, ctx->in_props.as<hlc_session_tally>(), d_state, d_status, s);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out_state, d_state, n, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(out_status, d_status, n, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}

uint64_t hlc_synth_arena_bytes(uint64_t n_proposals, uint32_t votes_per_proposal) {
  return hlc::synth_arena_bytes(n_proposals, votes_per_proposal);
}

int hlc_synth_votes_device(hlc_ctx* ctx, uint64_t seed, uint64_t start_proposal, uint64_t n_proposals,
                           uint32_t votes_per_proposal, uint32_t expected_voters, int gossipsub,
                           const hlc_votes* out_votes, hlc_proposal* out_proposals, uint8_t* out_priv, void* stream) {
  if (!ctx || !out_votes) return set_err(HLC_EINVAL, "NULL argument");
  const uint64_t n = n_proposals * (uint64_t)votes_per_proposal;
  if (votes_per_proposal && n / votes_per_proposal != n_proposals) return set_err(HLC_EINVAL, "size overflow");
  if (out_votes->n != n) return set_err(HLC_EINVAL, "out_votes->n must be n_proposals * votes_per_proposal");
  if (n && (!out_votes->vote_id || !out_votes->proposal_id || !out_votes->timestamp || !out_votes->vote ||
            !out_votes->bytes || !out_votes->field_off || !out_votes->field_len || !out_proposals))
    return set_err(HLC_EINVAL, "NULL output array");
  if (out_votes->bytes_len < hlc::synth_arena_bytes(n_proposals, votes_per_proposal))
    return set_err(HLC_EINVAL, "out_votes->bytes smaller than hlc_synth_arena_bytes()");
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
  CHK(ensure_fbtab(ctx));
  hlc::launch_synth(seed, start_proposal, n_proposals, votes_per_proposal, expected_voters, gossipsub, out_votes,
                    out_proposals, out_priv, ctx->fbtab, s);
  HIPCHK(hipGetLastError());
  return 0;
}

int hlc_synth_byzantine_device(hlc_ctx* ctx, uint64_t seed, uint64_t start_proposal, uint64_t n_proposals,
                               uint32_t votes_per_proposal, const hlc_votes* votes, uint8_t* out_kind,
                               void* stream) {
  if (!ctx || !votes) return set_err(HLC_EINVAL, "NULL argument");
  const uint64_t n = n_proposals * (uint64_t)votes_per_proposal;
  if (votes_per_proposal && n / votes_per_proposal != n_proposals) return set_err(HLC_EINVAL, "size overflow");
  if (votes->n != n) return set_err(HLC_EINVAL, "votes->n must be n_proposals * votes_per_proposal");
  if (n && (!out_kind || !votes->bytes || !votes->field_off || !votes->field_len || !votes->timestamp ||
            !votes->proposal_id || !votes->vote_id || !votes->vote))
    return set_err(HLC_EINVAL, "NULL vote / output array");
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
  CHK(ensure_fbtab(ctx));
  CHK(ctx->byz_key.ensure(n * 8 + 8));
  hlc::launch_synth_byzantine(seed, start_proposal, n_proposals, votes_per_proposal, votes, out_kind,
                              ctx->byz_key.as<uint64_t>(), ctx->fbtab, s);
  HIPCHK(hipGetLastError());
  return 0;
}

int hlc_eth_address_batch(hlc_ctx* ctx, uint64_t n, const uint8_t* priv32, uint8_t* out_addr20) {
  if (!ctx || (n && (!priv32 || !out_addr20))) return set_err(HLC_EINVAL, "NULL argument");
  if (!n) return 0;
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = ctx->stream;
  CHK(ensure_fbtab(ctx));
  CHK(upload(ctx->in_priv, priv32, n * 32, s));
  CHK(ctx->out_rec.ensure(n * 20 + 20));
  hlc::launch_address(n, ctx->in_priv.as<uint8_t>(), ctx->fbtab, ctx->out_rec.as<uint8_t>(), s);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out_addr20, ctx->out_rec.p, n * 20, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}

int hlc_eth_sign_batch(hlc_ctx* ctx, uint64_t n, const uint8_t* priv32, const uint8_t* bytes, uint64_t bytes_len,
                       const uint64_t* payload_off, const uint32_t* payload_len, uint8_t* out_sig65) {
  if (!ctx || (n && (!priv32 || !payload_off || !payload_len || !out_sig65)))
    return set_err(HLC_EINVAL, "NULL argument");
  for (uint64_t i = 0; i < n; ++i)
    if (payload_off[i] + payload_len[i] > bytes_len) return set_err(HLC_EINVAL, "payload outside the byte arena");
  if (!n) return 0;
  std::lock_guard<std::mutex> lk(ctx->mu);
  CHK(activate(ctx));
  hipStream_t s = ctx->stream;
  CHK(ensure_fbtab(ctx));
  CHK(upload(ctx->in_bytes, bytes, bytes_len, s));
  CHK(upload(ctx->in_off2, payload_off, n, s));
  CHK(upload(ctx->in_len2, payload_len, n, s));
  CHK(upload(ctx->in_priv, priv32, n * 32, s));
  CHK(run_prehash(ctx, nullptr, n, hlc::MSG_PAYLOAD, ctx->in_bytes.as<uint8_t>(), ctx->in_off2.as<uint64_t>(),
                  ctx->in_len2.as<uint32_t>(), s));
  CHK(ctx->out_misc.ensure(n * 65 + 65));
  hlc::launch_sign(n, ctx->in_priv.as<uint8_t>(), ctx->kec_dig.as<uint32_t>(), ctx->fbtab,
                   ctx->out_misc.as<uint8_t>(), s);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out_sig65, ctx->out_misc.p, n * 65, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}

}  // extern "C"
