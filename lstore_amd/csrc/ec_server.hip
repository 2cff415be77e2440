// ec_server.hip -- the stripe server: a persistent, self-retiring gfx950 kernel that serves
// small zero-copy encode / decode requests posted by host threads (SURVEY.md §2 caller loop:
// LStore calls plan->encode_block once per stripe, segment/jerasure.c:1847, from up to 300 pool
// threads).  A request part is one column block of one stripe; its descriptor and its chunks
// live in page-locked host memory (or the caller's own page-locked buffers), and the serving
// workgroup reads and writes them over PCIe -- no DMA, no launch per call.
//
// Protocol (two 64-byte lines per workgroup, so one wave-wide PCIe read polls all its slots):
//   host   writes desc[s], then post[g][i] = n  (n: the slot's next sequence number)
//   server sees post != served, acquires, copies desc (and the coefficient cells) into LDS,
//          computes, releases at system scope, writes done[s] = n
//   host   spins on done[s] == n, copies the outputs out, frees the slot
// post[g][31] is the stop word.  The kernel exits when every workgroup has been idle for
// idle_ticks (a collective vote, below) or when the stop word is set -- every wave reaches
// one of them -- and the host relaunches it on demand.  It runs on its own high-priority stream: such a stream has a hardware queue of its
// own, so the parked kernel never holds up other streams' packets (tools/probes/queue_probe.hip,
// profiles/r02_queue_probe.txt).
#include "ec_kernels_impl.h"
#include "ec_server.h"

namespace lsec {

namespace {

__device__ __forceinline__ uint32_t sys_load(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one column block of one stripe, bytewise GF(2^8) (RS / r6 / raid4 / XOR-only decodes):
// each lane owns 16 B columns, inputs in groups of 8 loads in flight
template <int R>
__device__ void srv_bytewise(const SrvDesc &d, const CoefCell *cl) {
  const int K = static_cast<int>(d.K);
  const int64_t C = static_cast<int64_t>(d.size);
  for (int64_t col = threadIdx.x * 16; col < C; col += kBlock * 16) {
    const bool whole = col + 16 <= C;  // else exactly 8 bytes remain (C % 8 == 0)
    u32x4 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0u;
    for (int j0 = 0; j0 < K; j0 += 8) {
      u32x4 v[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        v[jj] = 0u;
        if (j0 + jj < K) {
          const uint64_t p = d.in[j0 + jj] + col;
          if (whole) {
            v[jj] = *gptr<u32x4>(p);
          } else {
            const u32x2 h = *gptr<u32x2>(p);
            v[jj].x = h.x;
            v[jj].y = h.y;
          }
        }
      }
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        if (j0 + jj >= K) break;
        const u32x4 ia = v[jj] & 0x07070707u, ib = (v[jj] >> 3) & 0x07070707u, ic = (v[jj] >> 6) & 0x03030303u;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const CoefCell &c = cl[r * K + j0 + jj];
          const uint32_t t[6] = {c.ta_lo, c.ta_hi, c.tb_lo, c.tb_hi, c.tc_lo, c.tc_hi};
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[r][e] = gf_mul_acc(acc[r][e], ia[e], ib[e], ic[e], t);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t q = d.out[r] + col;
      if (whole) {
        *gptr_w<u32x4>(q) = acc[r];
      } else {
        u32x2 h;
        h.x = acc[r].x;
        h.y = acc[r].y;
        *gptr_w<u32x2>(q) = h;
      }
    }
  }
}

// one block of whole super-packets of one stripe, bit-sliced GF(2^8) (Cauchy): as
// k_gf8_bitsliced, with 4 inputs x 8 packet words in flight per lane
template <int R>
__device__ void srv_bitsliced(const SrvDesc &d, const CoefCell *cl) {
  const int K = static_cast<int>(d.K);
  const uint32_t P = d.packet;
  const uint32_t col_bytes = static_cast<uint32_t>(d.size / 8);
  for (uint32_t colb = threadIdx.x * 4; colb < col_bytes; colb += kBlock * 4) {
    const uint32_t sp = colb / P;
    const uint64_t off = static_cast<uint64_t>(sp) * 8 * P + (colb - sp * P);
    uint32_t acc[R][8];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int x = 0; x < 8; ++x) acc[r][x] = 0u;
    for (int j0 = 0; j0 < K; j0 += 4) {
      uint32_t e[4][8];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int x = 0; x < 8; ++x) e[jj][x] = j0 + jj < K ? *gptr<uint32_t>(d.in[j0 + jj] + off + x * P) : 0u;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        if (j0 + jj >= K) break;
        uint32_t c[R], cm = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          c[r] = cl[r * K + j0 + jj].coef;
          cm |= c[r];
        }
#pragma unroll
        for (int b = 0; b < 8; ++b) {
#pragma unroll
          for (int r = 0; r < R; ++r)
            if ((c[r] >> b) & 1u)
#pragma unroll
              for (int x = 0; x < 8; ++x) acc[r][x] ^= e[jj][x];
          if ((cm >> (b + 1)) == 0) break;
          const uint32_t top = e[jj][7];  // e <- 2e in bit-sliced form (x^8 = x^4 + x^3 + x^2 + 1)
          e[jj][7] = e[jj][6];
          e[jj][6] = e[jj][5];
          e[jj][5] = e[jj][4];
          e[jj][4] = e[jj][3] ^ top;
          e[jj][3] = e[jj][2] ^ top;
          e[jj][2] = e[jj][1] ^ top;
          e[jj][1] = e[jj][0];
          e[jj][0] = top;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int x = 0; x < 8; ++x) *gptr_w<uint32_t>(d.out[r] + off + x * P) = acc[r][x];
  }
}

template <int R>
__device__ void srv_serve(const SrvDesc &d, const CoefCell *cl) {
  if (d.kind == kSrvBytewise) srv_bytewise<R>(d, cl);
  else srv_bitsliced<R>(d, cl);
}

__global__ __launch_bounds__(kBlock) void k_stripe_server(SrvArgs a) {
  __shared__ SrvDesc d;
  __shared__ CoefCell cl[kSrvMaxR * kSrvMaxK];
  __shared__ uint32_t served[32];
  __shared__ int pick, quit, last_pick, voted;
  __shared__ uint32_t pick_val;
  __shared__ uint64_t idle_since;
  const int g = blockIdx.x;
  SrvShared *sh = a.shared;
  if (threadIdx.x < kSrvSlotsPerWG) served[threadIdx.x] = sys_load(&sh->done[srv_slot(g, threadIdx.x)][0]);
  if (threadIdx.x == 0) {
    last_pick = kSrvSlotsPerWG - 1;
    voted = 0;
    idle_since = wall_clock64();
  }
  __syncthreads();
  for (;;) {
    if (threadIdx.x < 64) {  // wave 0 polls this workgroup's line
      const int lane = threadIdx.x;
      const uint32_t v = lane < 32 ? sys_load(&sh->post[g][lane]) : 0u;
      // a.hold (test hook, lsec_test_server_hold): serve nothing, as a server that never answers
      const bool ready = lane < kSrvSlotsPerWG && v != served[lane] && !a.hold;
      const uint64_t m = __ballot(ready);
      const uint32_t stop = __shfl(v, kSrvSlotsPerWG);
      // round robin: the first ready slot after the last one served, so slots that other
      // threads keep re-posting cannot starve a higher one
      const uint64_t after = m & ~((2ull << last_pick) - 1);
      const uint64_t pool = after ? after : m;
      int first = pool ? __ffsll(static_cast<unsigned long long>(pool)) - 1 : -1;
      const uint32_t val = __shfl(v, first < 0 ? 0 : first);
      if (lane == 0) {
        int q = stop != 0;
        // The stop word is final: from the poll that sees it, nothing more is picked, so the
        // launch leaves after at most the part each workgroup is serving now, however busy the
        // posting threads keep the slots.  What is still posted waits for the next launch, which
        // reloads served[] from done[] (the host cancels the stopping call's own parts).
        if (q) first = -1;
        if (first >= 0 && voted) {
          // work again: take back the idle vote before serving -- unless the count is complete.
          // Retirement is a one-way latch: once every workgroup has voted, a workgroup that has
          // seen the full count may already have left (stranding its slots), so nobody may take
          // a vote back; this one leaves too and the post waits for the next launch, which
          // reloads served[] from done[] (a compare-and-swap refuses at kSrvWG).
          int cur = __hip_atomic_fetch_add(a.votes, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          while (cur < kSrvWG &&
                 !__hip_atomic_compare_exchange_strong(a.votes, &cur, cur - 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)) {
          }
          if (cur >= kSrvWG) {
            first = -1;
            q = 1;
          } else {
            voted = 0;
          }
        }
        if (first >= 0) {
          last_pick = first;
        } else if (!q) {
          // Exit is collective: a workgroup that left on its own would strand its slots while
          // the rest keep the kernel (and so the host's relaunch) waiting.  Idle workgroups
          // vote; all leave once every one has voted.  The count is read by an atomic
          // read-modify-write, coherent across the XCDs' L2s (a plain or relaxed-load time
          // stamp of "last work" can be stale in one XCD's L2 and let its workgroups leave).
          if (!voted && wall_clock64() - idle_since > a.idle_ticks) {
            __hip_atomic_fetch_add(a.votes, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            voted = 1;
          }
          if (voted && __hip_atomic_fetch_add(a.votes, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= kSrvWG) q = 1;
        }
        pick = first;
        pick_val = val;
        quit = q;
      }
    }
    __syncthreads();
    if (pick < 0) {
      if (quit) break;
      __builtin_amdgcn_s_sleep(16);
      __syncthreads();  // nobody rewrites pick / quit before every wave has read them
      continue;
    }
    const int s = srv_slot(g, pick);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the descriptor was written before the post
    {  // descriptor: lane-varying vector loads (page-locked host memory) into LDS
      const uint32_t *src = reinterpret_cast<const uint32_t *>(&sh->desc[s]);
      uint32_t *dst = reinterpret_cast<uint32_t *>(&d);
      for (uint32_t i = threadIdx.x; i < sizeof(SrvDesc) / 4; i += kBlock) dst[i] = sys_load(src + i);
    }
    __syncthreads();
    {  // the R x K coefficient cells of this request (device memory) into LDS, coherent loads:
       // a plan's image may sit where a destroyed plan's was while this kernel runs
      const uint32_t *src = reinterpret_cast<const uint32_t *>(d.cells);
      const uint32_t n = d.R * d.K * (sizeof(CoefCell) / 4), row = d.K * (sizeof(CoefCell) / 4),
                     stride = d.cstride * (sizeof(CoefCell) / 4);
      uint32_t *dst = reinterpret_cast<uint32_t *>(cl);
      for (uint32_t i = threadIdx.x; i < n; i += kBlock)
        dst[i] = __hip_atomic_load(src + (i / row) * stride + (i % row), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    switch (d.R) {
      case 1: srv_serve<1>(d, cl); break;
      case 2: srv_serve<2>(d, cl); break;
      case 3: srv_serve<3>(d, cl); break;
      case 4: srv_serve<4>(d, cl); break;
      case 5: srv_serve<5>(d, cl); break;
      case 6: srv_serve<6>(d, cl); break;
      case 7: srv_serve<7>(d, cl); break;
      default: srv_serve<8>(d, cl); break;
    }
    __threadfence_system();  // every output byte is out before the done flag
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_store(&sh->done[s][0], pick_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      served[pick] = pick_val;
      idle_since = wall_clock64();
    }
    __syncthreads();
  }
}

}  // namespace

hipError_t launch_stripe_server(const SrvArgs &a, hipStream_t st) {
  if (!a.shared || !a.votes) return hipErrorInvalidValue;
  return launch_kernel(&k_stripe_server, dim3(kSrvWG), dim3(kBlock), st, a);
}

}  // namespace lsec
