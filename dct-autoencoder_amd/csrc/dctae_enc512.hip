// k_enc512: the 512^2 encode's row and column passes in ONE persistent launch
// whose row -> column hand-off of the intermediate T stays inside one XCD,
// so T (2.75 MB per image) is written to and read from that XCD's L2 (and
// the Infinity Cache behind it) instead of making an HBM round trip between
// two launches (SURVEY §7 hard part 2; reference util.py:333-334: dct_2d =
// the row DCT, then the column DCT of its result).
//
// Work per image: 32 row items (16 rows each: rows512_item, dctae_rows512.h)
// then 96 column items ((channel, tile column) x 448 kept rows: the cols7
// transform + exact-threshold LFQ epilogue, dctae_spec512.h).  Every block
// reads its XCD's id (HW_REG_XCC_ID) at run time and takes items from that
// XCD's queue only, so producer and consumer of a T slot always share an L2;
// nothing depends on how the dispatcher places blocks (an XCD without blocks
// simply claims no images).
//
// Queue of XCD x (positions from its head counter), L = kLag:
//   segments 0 .. L - 1:   R(k) x 32
//   segment k >= L:        R(k) x 32, then C(k - L) x 96
// Segment k's image is claimed from the global image counter kAhead segments
// early, by the block that takes R(k - kAhead) item 0 (R(0, 0) claims
// segments 0 .. kAhead), each claim after segment k - 1's is published (so
// claims are monotone in k: once a segment gets no image, no later one does).
// Claiming at use instead stalled the segment's 31 other row items behind
// the claimer's previous item.
// L images are in flight per XCD: one image's rows alone take a block's item
// time (~26 us), so column items of the image just finished would wait.
// T slot of segment k: k % S (S = L + 2 per XCD).  Waits (every one on an
// item at a LOWER queue position, so the lowest unfinished item can always
// run: no deadlock, whatever the residency; a block holds at most one
// taken-ahead item, which is never lower than its current one):
//   R(k)     waits for C(k - S) done (its slot's previous reader);
//   C(k)     waits for R(k) done (all 32 row items of its image).
// Hand-off (same XCD, one L2): producer plain T stores -> every wave
// s_waitcnt vmcnt(0) -> barrier -> one agent-scope atomic add; consumer polls
// the counter with relaxed agent-scope (sc1) loads and reads T with sc1 buffer
// loads (L2-served, never a stale L1 line).  Every spin is bounded: on time
// out the block sets error bit 32 and leaves (dctae_check_device_errors).
#include "dctae_launch.h"
#include "dctae_rows512.h"
#include "dctae_spec512.h"

namespace dctae {

namespace {

constexpr int kRowItems = 32;                    // 16-row items per image
constexpr int kColItems = 96;                    // (channel, tile column) items per image
constexpr int kSeg = kRowItems + kColItems;
#ifndef DCTAE_ENC_LAG
#define DCTAE_ENC_LAG 2
#endif
constexpr int kLag = DCTAE_ENC_LAG;              // column items of image k follow the row items of image k + kLag
constexpr int kSlots = kLag + 2;                 // T slots per XCD
constexpr int kAhead = 2;                        // R(k, 0) claims the image of segment k + kAhead
#ifndef DCTAE_ENC_PREL
#define DCTAE_ENC_PREL 0                         // producer agent-scope release before the row-done add
#endif
#ifndef DCTAE_ENC_CACQ
#define DCTAE_ENC_CACQ 0                         // consumer agent-scope acquire after the row-done poll
#endif
#ifndef DCTAE_ENC_RESERVE
#define DCTAE_ENC_RESERVE 1                      // take the next position while the current item runs
#endif
constexpr int kKW = 448, kH = 512;
constexpr int64_t kSlotFloats = 3ll * kH * kKW;  // one image's T
constexpr unsigned kNone = 0x7fffffffu;          // published "no image" (claims start at 1)
constexpr uint64_t kSpinTicks = 50000000ull;    // bounded waits: 0.5 s of s_memrealtime (100 MHz)

// sync block (unsigned words, zeroed per call): [0] image claim counter,
// [32 (x + 1)] head of XCD x (own 128-byte lines), then
// img[x][seg] (claimed image + 1, or kNone), rdone[n], cdone[n]
constexpr int kHeadBase = 32;
constexpr int kImgBase = 32 * 9;

union EncU {
  Rows512Xch rows;
  Cols7Lds cols;
};

struct EncLds {
  EncU u;
  Rows512Tab rt;
  float4 post4[257];
  float2 tw_s[256];
  float sbias[32];
  int item[4];
};

__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
#ifdef DCTAE_ENC_RMWPOLL
  return __hip_atomic_fetch_add(const_cast<unsigned*>(p), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

// one lane: poll *p until pred holds (bounded in wall time; false on time out)
template <class Pred>
__device__ __forceinline__ bool spin_until(const unsigned* p, Pred pred, unsigned& v) {
  v = ld_agent(p);
  if (pred(v)) return true;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    __builtin_amdgcn_s_sleep(2);
    v = ld_agent(p);
    if (pred(v)) return true;
    if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) return false;
  }
}

// queue position -> (row item?, segment of its image k, item index i)
__device__ __forceinline__ void decode_pos(int p, bool& is_row, int& k, int& i) {
  if (p < kLag * kRowItems) {
    is_row = true, k = p / kRowItems, i = p % kRowItems;
    return;
  }
  const int q = p - kLag * kRowItems, r = q % kSeg;
  k = q / kSeg + kLag;
  is_row = r < kRowItems;
  i = is_row ? r : r - kRowItems;
  if (!is_row) k -= kLag;   // C items of segment k serve image k - kLag
}

#ifdef DCTAE_ENC_CHECK
// debug builds: protocol invariants (claims per image, slot owners)
__device__ unsigned g_chk_claims[1 << 16];
__device__ unsigned g_chk_owner[8][8];
__device__ unsigned g_chk_bad[4];
#endif

#ifdef DCTAE_ENC_STATS
// profiling builds (-DDCTAE_ENC_STATS): per-XCD item timing, printed by the
// last block to leave: [0] blocks [1] row items [2] column items [3] wait
// ticks [4] row ticks [5] column ticks [6] block lifetime ticks [7] row-item wait
// ticks (100 MHz)
__device__ unsigned long long g_enc_st[8][8];
__device__ unsigned g_enc_st_left;
#endif

// take the next queue position of XCD x (one lane).  A position that is a
// segment's first row item R(k, 0) claims the image of segment k + kAhead
// right here (R(0, 0): segments 0 .. kAhead), after segment k + kAhead - 1's
// claim is published -- by whoever took R(k - 1, 0), also at its take, so the
// claim chain advances at dequeue speed and never waits on item processing.
// false: a wait timed out.
__device__ __forceinline__ bool take_pos(unsigned* head, unsigned* sync, unsigned* img_tab, int n_img, int max_seg,
                                         int& p) {
  p = (int)__hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  bool is_row;
  int k, i;
  decode_pos(p, is_row, k, i);
  if (!is_row || i != 0) return true;
  for (int kc = k == 0 ? 0 : k + kAhead; kc <= k + kAhead && kc < max_seg; ++kc) {
    unsigned prev = 1, got = kNone;
    if (kc > 0 && !spin_until(img_tab + kc - 1, [](unsigned v) { return v != 0u; }, prev)) return false;
    if (prev != kNone) {
      const unsigned n = __hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      got = n < (unsigned)n_img ? n + 1 : kNone;
#ifdef DCTAE_ENC_CHECK
      if (got != kNone) printf("CLAIM %u %u %d %u\n", n, (unsigned)(head - sync) / kHeadBase - 1, kc,
                               __builtin_amdgcn_s_getreg((3 << 11) | 20));
      if (got != kNone && atomicAdd(&g_chk_claims[n], 1u) != 0) {
        atomicAdd(&g_chk_bad[0], 1u);
        printf("CHK double claim image %u seg %d\n", n, kc);
      }
#endif
    }
    __hip_atomic_store(img_tab + kc, got, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return true;
}

}  // namespace

__global__ __launch_bounds__(256, 3) void k_enc512(const ImgDesc* __restrict__ imgs, int n_img,
                                               const float* __restrict__ rgb, float* __restrict__ tslots,
                                               const float2* __restrict__ tw, const float2* __restrict__ post,
                                               ColorMats cm, EncParams ep, TokenSinks sk, unsigned* __restrict__ sync,
                                               int max_seg, int* __restrict__ err) {
  __shared__ EncLds L;
  const int tid = threadIdx.x;
  rows512_tables(L.rt, tw, post);
  {
    const float4* p4 = reinterpret_cast<const float4*>(post);
    for (int i = tid; i < 257; i += 256) L.post4[i] = p4[i];
    L.tw_s[tid] = tw[tid];
  }
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
#ifdef DCTAE_ENC_ONEQ
  const int x = 0 * (int)(xcc & 7);   // debug: one queue for the whole chip (needs the agent fences)
#else
  const int x = (int)(xcc & 7);
#endif
  unsigned* head = sync + kHeadBase * (x + 1);
  unsigned* img_tab = sync + kImgBase + (size_t)x * max_seg;
  unsigned* rdone = sync + kImgBase + (size_t)8 * max_seg;
  unsigned* cdone = rdone + n_img;
  float* tx = tslots + (int64_t)x * kSlots * kSlotFloats;

  // item state in LDS: [0] current position, [1] the taken-ahead position,
  // [2] image of the current item (or kNone), [3] abort flag
  if (tid == 0) {
    int p0;
    L.item[3] = take_pos(head, sync, img_tab, n_img, max_seg, p0) ? 0 : 1;
    L.item[0] = p0;
  }
#ifdef DCTAE_ENC_STATS
  unsigned long long st[8] = {1, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long t_born = __builtin_amdgcn_s_memrealtime();
  unsigned long long t_a = 0, t_b = 0;
#endif
  for (;;) {
    __syncthreads();   // tables (first pass); the previous item's LDS use is over
#ifdef DCTAE_ENC_STATS
    if (tid == 0) t_a = __builtin_amdgcn_s_memrealtime();
#endif
    const int p = L.item[0];
    bool is_row;
    int k, i;
    decode_pos(p, is_row, k, i);
    if (tid == 0 && !L.item[3]) {
      unsigned img = kNone;
      bool ok = true;
#if DCTAE_ENC_RESERVE
      // take the next position now: the atomic's latency hides behind this item
      {
        int pn;
        ok = take_pos(head, sync, img_tab, n_img, max_seg, pn);
        L.item[1] = pn;
      }
#endif
      if (ok) {
        if (k >= max_seg) img = kNone;
        else ok = spin_until(img_tab + k, [](unsigned v) { return v != 0u; }, img);
      }
      if (ok && img != kNone) {
        const unsigned n = img - 1;
        unsigned v;
#ifdef DCTAE_ENC_NOWAIT
        if (false) {   // profiling build: no dependency waits (wrong outputs)
#else
        if (is_row) {
#endif
          // the slot's previous reader: segment k - S's 96 column items
          if (k >= kSlots) {
            const unsigned pimg = ld_agent(img_tab + k - kSlots);   // published (earlier claim)
            if (pimg != kNone) ok = spin_until(cdone + (pimg - 1), [](unsigned c) { return c >= (unsigned)kColItems; }, v);
          }
        } else {
#ifndef DCTAE_ENC_NOWAIT
          ok = spin_until(rdone + n, [](unsigned c) { return c >= (unsigned)kRowItems; }, v);
#endif
        }
      }
      if (!ok) {
        atomicOr(err, 32);
        L.item[3] = 1;
#ifdef DCTAE_ENC_DEBUG
        printf("k_enc512 wait timed out: xcc %d block %d pos %d (%s k %d i %d) img %u rdone %u cdone %u claim %u\n",
               x, (int)blockIdx.x, p, is_row ? "R" : "C", k, i, img,
               img != kNone && img ? ld_agent(rdone + img - 1) : 0u, img != kNone && img ? ld_agent(cdone + img - 1) : 0u,
               ld_agent(sync));
#endif
      }
      L.item[2] = (int)img;
#if DCTAE_ENC_CACQ
      if (!is_row && ok && img != kNone) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
#endif
    }
    __syncthreads();
#ifdef DCTAE_ENC_STATS
    if (tid == 0) {
      t_b = __builtin_amdgcn_s_memrealtime();
      st[3] += t_b - t_a;
      if (is_row) st[7] += t_b - t_a;
    }
#endif
    if (L.item[3]) break;   // a hand-off timed out (error bit 32)
    const unsigned img = (unsigned)L.item[2];
    if (img == kNone) {
      // a column item without an image: every later position is empty too
      // (claims are monotone; a taken-ahead position made its claim at take)
      if (!is_row) break;
    } else {
      const int n = (int)img - 1;
      const ImgDesc d = imgs[n];
      float* T = tx + (int64_t)(k % kSlots) * kSlotFloats;
#ifdef DCTAE_ENC_CHECK
      if (tid == 0) {
        const int sl = k % kSlots;
        if (is_row) {
          const unsigned prev = atomicExch(&g_chk_owner[x][sl], img);
          if (prev != 0 && prev != img && ld_agent(cdone + prev - 1) != (unsigned)kColItems) {
            atomicAdd(&g_chk_bad[1], 1u);
            printf("CHK slot reuse: xcd %d seg %d slot %d img %u prev %u prev-cdone %u\n", x, k, sl, img, prev,
                   ld_agent(cdone + prev - 1));
          }
        } else {
          const unsigned own = __hip_atomic_load(&g_chk_owner[x][sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const unsigned rd = ld_agent(rdone + n);
          if (own != img || rd != (unsigned)kRowItems) {
            atomicAdd(&g_chk_bad[2], 1u);
            printf("CHK col item: xcd %d seg %d slot %d img %u owner %u rdone %u\n", x, k, sl, img, own, rd);
          }
        }
      }
#endif
      if (is_row) {
        rows512_item<0>(L.u.rows, L.rt, rgb + d.rgb_off, kH, 16 * i, T, (uint32_t)(kH * kKW * 4), cm);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's T stores reached the L2
        __syncthreads();
        if (tid == 0) {
#if DCTAE_ENC_PREL
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
          __hip_atomic_fetch_add(rdone + n, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        const int c = i >> 5, strip = i & 31;
        float2 thr_r[2][7];
        cols_thresholds<true>(d, c, strip, ep, thr_r, L.sbias);
        float va[16], vb[16];
        cols7_load<16>(d, c, strip, T, va, vb);
        cols7_compute<true>(d, c, strip, L.u.cols, va, vb, L.post4, L.tw_s, L.sbias, thr_r, ep, sk);
        __syncthreads();   // every wave's T loads have returned (their values were used)
        if (tid == 0) __hip_atomic_fetch_add(cdone + n, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#ifdef DCTAE_ENC_STATS
      if (tid == 0) {
        const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t_b;
        st[is_row ? 1 : 2] += 1;
        st[is_row ? 4 : 5] += dt;
      }
#endif
    }
    if (tid == 0) {
#if DCTAE_ENC_RESERVE
      L.item[0] = L.item[1];
#else
      int pn;
      if (!take_pos(head, sync, img_tab, n_img, max_seg, pn)) {
        atomicOr(err, 32);
        L.item[3] = 1;
      }
      L.item[0] = pn;
#endif
    }
  }
#ifdef DCTAE_ENC_STATS
  if (tid == 0) {
    st[6] = __builtin_amdgcn_s_memrealtime() - t_born;
    for (int e = 0; e < 8; ++e) atomicAdd(&g_enc_st[x][e], st[e]);
    __threadfence();
    if (atomicAdd(&g_enc_st_left, 1u) == gridDim.x - 1) {
      __threadfence();
      for (int xx = 0; xx < 8; ++xx) {
        unsigned long long v[8];
        for (int e = 0; e < 8; ++e) v[e] = atomicExch(&g_enc_st[xx][e], 0ull);
        const double b = v[0] ? (double)v[0] : 1.0;
        printf("enc512 xcd %d: blocks %llu rows %llu (%.1f us, wait %.2f) cols %llu (%.1f us, wait %.2f) life/block %.1f us\n",
               xx, v[0], v[1], v[1] ? v[4] / 100.0 / v[1] : 0.0, v[1] ? v[7] / 100.0 / v[1] : 0.0, v[2],
               v[2] ? v[5] / 100.0 / v[2] : 0.0, v[2] ? (v[3] - v[7]) / 100.0 / v[2] : 0.0, v[6] / 100.0 / b);
      }
      atomicExch(&g_enc_st_left, 0u);
    }
  }
#endif
}

size_t enc512_sync_words(int n_img) {
  const int max_seg = n_img + kLag + kAhead + 2;
  return (size_t)kImgBase + (size_t)8 * max_seg + 2 * (size_t)n_img;
}

size_t enc512_slot_bytes() { return (size_t)8 * kSlots * kSlotFloats * sizeof(float); }

int enc512_grid(int device) {
  static int cached[64] = {0};
  if (device >= 0 && device < 64 && cached[device]) return cached[device];
  int per_cu = 0, n_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_enc512, 256, 0) != hipSuccess || per_cu < 1) per_cu = 2;
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n_cu < 1)
    n_cu = 256;
  hipGetLastError();
  const int g = per_cu * n_cu;
  if (device >= 0 && device < 64) cached[device] = g;
  return g;
}

// imgs: n_img 512 x 512 images with qh = qw = 32 (Kw = Kh = 448) in one
// staging (tok_off); sync: enc512_sync_words(n_img) words, zeroed here;
// tslots: enc512_slot_bytes().  ep must carry the exact LFQ thresholds.
void launch_enc512(const ImgDesc* imgs, int n_img, const float* rgb, float* tslots, const float2* tw,
                   const float2* post, const ColorMats& cm, const EncParams& ep, const TokenSinks& sk, unsigned* sync,
                   int grid, int* err, hipStream_t s) {
  if (n_img <= 0) return;
  hipMemsetAsync(sync, 0, enc512_sync_words(n_img) * sizeof(unsigned), s);
  hipLaunchKernelGGL(k_enc512, dim3(grid), dim3(256), 0, s, imgs, n_img, rgb, tslots, tw, post, cm, ep, sk, sync,
                     n_img + kLag + kAhead + 2, err);
}

}  // namespace dctae
