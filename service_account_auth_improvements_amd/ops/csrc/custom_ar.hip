// One-shot all-reduce over peer-mapped HIP IPC buffers (C7 in SURVEY.md §2.8: the per-layer,
// per-token TP all-reduce of InferenceService decode with TP > 1).
//
// Decode all-reduces are tiny ([B, hidden] bf16: 16 KB at B = 1 for 70B) and sit on the
// token-latency critical path twice per layer, where a ring (RCCL) pays 2(N-1) link hops of
// latency.  On one MI355X node every GPU pair has its own xGMI link, so each rank can read
// every peer's copy directly and sum locally: ONE hop, one kernel, no host involvement.
//
// Buffer of each rank (hipExtMallocWithFlags(..., hipDeviceMallocUncached): the flags are
// polled by other GPUs and the data is read by them across xGMI, so nothing may sit in a
// non-coherent cache), exported with hipIpcGetMemHandle and opened by every peer:
//   [flags: 2 slots x MAXB blocks x MAXW ranks int32][epochs: MAXB int32][err: int32]
//   [data: 2 slots x slot_bytes]
// Call protocol, per block b (no grid-wide sync; blocks own disjoint chunks):
//   e = ++epoch[b] (block-private counter, so HIP-graph replays need no host epoch);
//   slot = e & 1; copy my chunk of x into data[slot];
//   release (system scope) -> write e into flags[slot][b][my_rank] of EVERY peer;
//   spin until flags[slot][b][p] == e for all p in my buffer -> acquire.  The wait is bounded
//   in WALL TIME (s_memrealtime, 100 MHz), by a budget the caller passes per call (the decode
//   engine a few seconds, a training communicator its process-group timeout): a late peer is
//   waited for, a dead one sets err and the kernel gives up instead of hanging the GPU;
//   out[chunk] = sum_p peer_p.data[slot][chunk], accumulated in fp32 in rank order, so every
//   rank produces bit-identical results.  out may be x (in place, like dist.all_reduce): a
//   block reads its chunk of x before the flag exchange and writes it after.
// Two slots suffice: to enter call e a block needs every peer's call-(e-1) flag, i.e. every
// peer block has finished reading call e-2's data from the slot being overwritten.
#include <cstring>

#include "common.h"

using namespace kf;

namespace car {
constexpr int MAXW = 8;        // ranks (one MI355X node)
constexpr int MAXB = 64;       // blocks (chunks) per call
constexpr int NT = 512;
constexpr long FLAG_BYTES = 2L * MAXB * MAXW * 4;
constexpr long EPOCH_OFF = FLAG_BYTES;
constexpr long ERR_OFF = EPOCH_OFF + MAXB * 4;
constexpr long DATA_OFF = 8192;  // header padded to 8 KB
constexpr double RT_HZ = 1e8;    // s_memrealtime ticks per second

// Wait until *f == e; false once `budget` ticks of the constant 100 MHz realtime counter
// have passed (a clock that does not move with the shader clock, so the budget is seconds).
__device__ __forceinline__ bool wait_flag(int* f, int e, unsigned long long budget) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != e) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > budget) return false;
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}
__host__ inline unsigned long long budget_ticks(double timeout_s) {
  return (unsigned long long)(std::max(timeout_s, 1e-3) * RT_HZ);
}

struct Peers {
  char* p[MAXW];
};

__device__ __forceinline__ int* flags(char* base, int slot, int b, int r) {
  return reinterpret_cast<int*>(base) + ((slot * MAXB + b) * MAXW + r);
}

template <int W>
__global__ __launch_bounds__(NT) void one_shot_ar_kernel(Peers peers, int rank, const bf16_t* x, bf16_t* out,
                                                         long n, long slot_bytes, unsigned long long budget) {
  __shared__ int e_sh;
  const int b = blockIdx.x, tid = threadIdx.x;
  char* mine = peers.p[rank];
  int* epoch = reinterpret_cast<int*>(mine + EPOCH_OFF) + b;
  if (tid == 0) e_sh = __hip_atomic_load(epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  const int e = e_sh, slot = e & 1;
  // chunk of 8-element (16 B) vectors owned by this block
  const long nv = n / 8, per = (nv + gridDim.x - 1) / gridDim.x;
  const long v0 = b * per, v1 = min(nv, v0 + per);
  u32x4* dst = reinterpret_cast<u32x4*>(mine + DATA_OFF + slot * slot_bytes);
  for (long v = v0 + tid; v < v1; v += NT) dst[v] = ld16(x + 8 * v);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid < W) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope: data before flag, for every GPU
    __hip_atomic_store(flags(peers.p[tid], slot, b, rank), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (!wait_flag(flags(mine, slot, b, tid), e, budget))
      __hip_atomic_store(reinterpret_cast<int*>(mine + ERR_OFF), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  for (long v = v0 + tid; v < v1; v += NT) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < W; ++p) {
      const u32x4 src = reinterpret_cast<const u32x4*>(peers.p[p] + DATA_OFF + slot * slot_bytes)[v];
      float f[8];
      unpack8(src, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    st16(out + 8 * v, pack8(acc));
  }
  if (tid == 0) __hip_atomic_store(epoch, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace car

// ==== two-shot reduce-scatter / all-gather for training-size TP messages (16-268 MB) ===========
// RCCL's ring moves an all-reduce over one link per hop; on a full xGMI mesh every rank can pull
// from all N-1 peers at once.  Two-shot: rank r owns chunk r (1/N of the tensor); phase 1 it
// reads chunk r from every peer's input and sums it (fp32, rank order -> every rank's result is
// bit-identical, and for N = 2 equal to one bf16 rounding of the exact sum, as RCCL's), phase 2
// every rank reads every peer's reduced chunk.  Each link carries 2 S / N per direction -- the
// all-reduce minimum -- and all N-1 links of a GPU carry it concurrently.
//   mode AR: input x[n] -> out[n] (sum)      mode RS: x[n] -> out[n/N] (own chunk of the sum)
//   mode AG: x[n/N] (own chunk) -> out[n] (concatenation in rank order)
// Buffer (uncached, IPC-exported, zeroed): [phase-1 flags | phase-2 flags: 2 slots x MAXB x MAXW
// int32 each][epochs MAXB][err][pad to 32 KB][in: 2 slots x slot_bytes][red: 2 slots x slot_bytes/N]
// Same per-block epoch / two-slot argument as the one-shot kernel: to enter call e a block has
// seen every peer's call-(e-1) phase-2 flag, so no peer still reads call e-2's slot.
// Every block's epoch advances once per call, so the communicator keeps ONE grid size for its
// life (parallel/custom_ar.py TwoShot) and issues its calls on ONE stream: then every in-flight
// block of every rank is in call k or k+1, and parity slots never collide.
namespace ts {
constexpr int MAXW = 8, MAXB = 128, NT = 512;
constexpr long FLAGS1 = 0, FLAGS2 = 2L * MAXB * MAXW * 4, EPOCH_OFF = 2 * FLAGS2, ERR_OFF = EPOCH_OFF + MAXB * 4;
constexpr long DATA_OFF = 32768;
static_assert(ERR_OFF + 4 <= DATA_OFF, "two-shot header");
enum Mode { AR = 0, RS = 1, AG = 2 };

__device__ __forceinline__ int* flag(char* base, long off, int slot, int b, int r) {
  return reinterpret_cast<int*>(base + off) + ((slot * MAXB + b) * MAXW + r);
}
// lanes 0..W-1: post e to every peer's flag (release first), then wait for every peer's flag
template <int W>
__device__ __forceinline__ void exchange(const car::Peers& P, int rank, long off, int slot, int b, int e, char* mine,
                                         unsigned long long budget) {
  const int tid = threadIdx.x;
  __syncthreads();
  if (tid < W) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(flag(P.p[tid], off, slot, b, rank), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (!car::wait_flag(flag(mine, off, slot, b, tid), e, budget))
      __hip_atomic_store(reinterpret_cast<int*>(mine + ERR_OFF), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
}

template <int W, int MODE>
__global__ __launch_bounds__(NT) void two_shot_kernel(car::Peers P, int rank, const bf16_t* x, bf16_t* out,
                                                      long n, long slot_bytes, unsigned long long budget) {
  __shared__ int e_sh;
  const int b = blockIdx.x, tid = threadIdx.x;
  char* mine = P.p[rank];
  int* epoch = reinterpret_cast<int*>(mine + EPOCH_OFF) + b;
  if (tid == 0) e_sh = __hip_atomic_load(epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  const int e = e_sh, slot = e & 1;
  const long red_bytes = slot_bytes / W;
  auto in_of = [&](int p) { return reinterpret_cast<u32x4*>(P.p[p] + DATA_OFF + slot * slot_bytes); };
  auto red_of = [&](int p) {
    return reinterpret_cast<u32x4*>(P.p[p] + DATA_OFF + 2 * slot_bytes + slot * red_bytes);
  };
  // this block's share of one chunk, in 16-byte vectors (chunk = n / W elements)
  const long cv = n / W / 8, per = (cv + gridDim.x - 1) / gridDim.x;
  const long v0 = b * per, v1 = min(cv, v0 + per);
  const u32x4* xin = reinterpret_cast<const u32x4*>(x);
  if (MODE != AG) {
    u32x4* mine_in = in_of(rank);
    for (int c = 0; c < W; ++c)
      for (long v = v0 + tid; v < v1; v += NT) mine_in[c * cv + v] = xin[c * cv + v];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    exchange<W>(P, rank, FLAGS1, slot, b, e, mine, budget);
    // phase 1: reduce my chunk over every peer's input (rank order)
    u32x4* red = red_of(rank);
    for (long v = v0 + tid; v < v1; v += NT) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      u32x4 src[W];
#pragma unroll
      for (int p = 0; p < W; ++p) src[p] = in_of(p)[rank * cv + v];
#pragma unroll
      for (int p = 0; p < W; ++p) {
        float f[8];
        unpack8(src[p], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f[j];
      }
      const u32x4 r = pack8(acc);
      if (MODE == AR) red[v] = r;
      reinterpret_cast<u32x4*>(out)[(MODE == AR ? rank * cv : 0) + v] = r;
    }
    if (MODE == AR) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    u32x4* red = red_of(rank);
    for (long v = v0 + tid; v < v1; v += NT) {
      red[v] = xin[v];
      reinterpret_cast<u32x4*>(out)[rank * cv + v] = xin[v];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (MODE != RS) {
    exchange<W>(P, rank, FLAGS2, slot, b, e, mine, budget);
    // phase 2: every peer's reduced chunk
    for (long v = v0 + tid; v < v1; v += NT) {
      u32x4 src[W];
#pragma unroll
      for (int p = 0; p < W; ++p) src[p] = red_of(p)[v];
#pragma unroll
      for (int p = 0; p < W; ++p)
        if (p != rank) reinterpret_cast<u32x4*>(out)[p * cv + v] = src[p];
    }
  } else {
    // RS posts phase 2 too (without reading anything): the slot-reuse argument needs every
    // call's phase-2 flags
    exchange<W>(P, rank, FLAGS2, slot, b, e, mine, budget);
  }
  if (tid == 0) __hip_atomic_store(epoch, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int W>
void launch_two_shot(int mode, int blocks, hipStream_t st, const car::Peers& P, int rank, const bf16_t* x, bf16_t* o,
                     long n, long slot_bytes, unsigned long long bt) {
  if (mode == AR) hipLaunchKernelGGL((two_shot_kernel<W, AR>), dim3(blocks), dim3(NT), 0, st, P, rank, x, o, n, slot_bytes, bt);
  else if (mode == RS) hipLaunchKernelGGL((two_shot_kernel<W, RS>), dim3(blocks), dim3(NT), 0, st, P, rank, x, o, n, slot_bytes, bt);
  else hipLaunchKernelGGL((two_shot_kernel<W, AG>), dim3(blocks), dim3(NT), 0, st, P, rank, x, o, n, slot_bytes, bt);
}
}  // namespace ts

using namespace car;

extern "C" {

long kf_car_header_bytes() { return DATA_OFF; }

// Allocate this rank's uncached, IPC-exportable buffer (zeroed); handle: 64-byte hipIpcMemHandle_t.
int kf_car_alloc(long slot_bytes, void** ptr, void* handle) {
  const long bytes = DATA_OFF + 2 * slot_bytes;
  if (hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached) != hipSuccess) return 1;
  if (hipMemset(*ptr, 0, bytes) != hipSuccess) return 2;
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, *ptr) != hipSuccess) return 4;
  std::memcpy(handle, &h, sizeof(h));
  return 0;
}

int kf_car_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  return hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess ? 0 : 1;
}

int kf_car_close(void* ptr) { return hipIpcCloseMemHandle(ptr) == hipSuccess ? 0 : 1; }
int kf_car_free(void* ptr) { return hipFree(ptr) == hipSuccess ? 0 : 1; }

// ptrs: world device pointers (own buffer at index rank); x/out: n bf16 (n % 8 == 0,
// 2 * n <= slot_bytes; out == x allowed); timeout_s: how long a block waits for a peer before
// it sets the error word.  Returns non-zero on a bad shape (nothing launched).
int kf_car_allreduce(void* const* ptrs, int world, int rank, const void* x, void* out, long n, long slot_bytes,
                     int blocks, double timeout_s, hipStream_t st) {
  if (world < 1 || world > MAXW || rank < 0 || rank >= world || n % 8 || 2 * n > slot_bytes) return 1;
  if (((uintptr_t)x | (uintptr_t)out) & 15) return 2;
  blocks = std::max(1, std::min(blocks, MAXB));
  Peers P{};
  for (int i = 0; i < world; ++i) P.p[i] = static_cast<char*>(ptrs[i]);
  auto X = static_cast<const bf16_t*>(x);
  auto O = static_cast<bf16_t*>(out);
  const unsigned long long bt = budget_ticks(timeout_s);
  switch (world) {
    case 1: hipLaunchKernelGGL(one_shot_ar_kernel<1>, dim3(blocks), dim3(NT), 0, st, P, rank, X, O, n, slot_bytes, bt); break;
    case 2: hipLaunchKernelGGL(one_shot_ar_kernel<2>, dim3(blocks), dim3(NT), 0, st, P, rank, X, O, n, slot_bytes, bt); break;
    case 4: hipLaunchKernelGGL(one_shot_ar_kernel<4>, dim3(blocks), dim3(NT), 0, st, P, rank, X, O, n, slot_bytes, bt); break;
    case 8: hipLaunchKernelGGL(one_shot_ar_kernel<8>, dim3(blocks), dim3(NT), 0, st, P, rank, X, O, n, slot_bytes, bt); break;
    default: return 3;
  }
  KF_CHECK_LAUNCH();
  return 0;
}

long kf_ts_header_bytes() { return ts::DATA_OFF; }

// this rank's two-shot buffer: header + 2 input slots + 2 reduced-chunk slots
int kf_ts_alloc(long slot_bytes, int world, void** ptr, void* handle) {
  if (world < 1 || world > ts::MAXW) return 5;
  const long bytes = ts::DATA_OFF + 2 * slot_bytes + 2 * (slot_bytes / world);
  if (hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached) != hipSuccess) return 1;
  if (hipMemset(*ptr, 0, bytes) != hipSuccess) return 2;
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, *ptr) != hipSuccess) return 4;
  std::memcpy(handle, &h, sizeof(h));
  return 0;
}

// mode 0 all-reduce (x[n] -> out[n]), 1 reduce-scatter (x[n] -> out[n/world]), 2 all-gather
// (x[n/world] -> out[n]); n is the FULL element count; n % (8 world) == 0, 2n <= slot_bytes.
int kf_ts_run(int mode, void* const* ptrs, int world, int rank, const void* x, void* out, long n, long slot_bytes,
              int blocks, double timeout_s, hipStream_t st) {
  if (world < 1 || world > ts::MAXW || rank < 0 || rank >= world || mode < 0 || mode > 2) return 1;
  if (n % (8L * world) || 2 * n > slot_bytes || slot_bytes % (16L * world)) return 1;
  if (((uintptr_t)x | (uintptr_t)out) & 15) return 2;
  if (mode == ts::AR && x != out) return 3;              // in place, like dist.all_reduce
  blocks = std::max(1, std::min(blocks, ts::MAXB));
  Peers P{};
  for (int i = 0; i < world; ++i) P.p[i] = static_cast<char*>(ptrs[i]);
  auto X = static_cast<const bf16_t*>(x);
  auto O = static_cast<bf16_t*>(out);
  const unsigned long long bt = budget_ticks(timeout_s);
  switch (world) {
    case 1: ts::launch_two_shot<1>(mode, blocks, st, P, rank, X, O, n, slot_bytes, bt); break;
    case 2: ts::launch_two_shot<2>(mode, blocks, st, P, rank, X, O, n, slot_bytes, bt); break;
    case 4: ts::launch_two_shot<4>(mode, blocks, st, P, rank, X, O, n, slot_bytes, bt); break;
    case 8: ts::launch_two_shot<8>(mode, blocks, st, P, rank, X, O, n, slot_bytes, bt); break;
    default: return 4;
  }
  KF_CHECK_LAUNCH();
  return 0;
}

// Asynchronous read of the error word: queued on `st` (after the calls it must cover) into
// pinned host memory; the caller looks at it once an event after this copy has completed, so
// checking costs no host synchronisation.  The word is not cleared: once set, the
// communicator is out of step for good.
int kf_ts_error_async(void* own, int* host_pinned, hipStream_t st) {
  char* p = static_cast<char*>(own) + ts::ERR_OFF;
  return hipMemcpyAsync(host_pinned, p, 4, hipMemcpyDeviceToHost, st) == hipSuccess ? 0 : 1;
}

int kf_ts_error(void* own, hipStream_t st) {
  int v = 0;
  char* p = static_cast<char*>(own) + ts::ERR_OFF;
  if (hipMemcpyAsync(&v, p, 4, hipMemcpyDeviceToHost, st) != hipSuccess) return -1;
  if (hipStreamSynchronize(st) != hipSuccess) return -1;
  if (v) {
    const int z = 0;
    hipMemcpy(p, &z, 4, hipMemcpyHostToDevice);
  }
  return v;
}

// error word (1 = a peer never arrived within the spin budget); cleared by the read
int kf_car_error(void* own, hipStream_t st) {
  int v = 0;
  char* p = static_cast<char*>(own) + ERR_OFF;
  if (hipMemcpyAsync(&v, p, 4, hipMemcpyDeviceToHost, st) != hipSuccess) return -1;
  if (hipStreamSynchronize(st) != hipSuccess) return -1;
  if (v) {
    const int z = 0;
    hipMemcpy(p, &z, 4, hipMemcpyHostToDevice);
  }
  return v;
}
}
