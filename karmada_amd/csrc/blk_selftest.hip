// blk_selftest.hip — test-only library (libkp_blktest.so): checks every GpuBlk
// primitive (kp_blk.h) on the device against a host computation, for several
// workgroup sizes and seeded random inputs. Never linked into libkp.so.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "kp_blk.h"
#include "kp_pdq.h"
#include "kp_select.h"

using namespace kp;

namespace {
// out layout per block: [0] sum64 [1] min64 [2] max64 [3] minu64 [4] and64 [5] or64
// [6] sum2.x [7] sum2.y [8] maxsum.max [9] maxsum.sum [10] any [11] bcast
// [12] andor.and [13] andor.or [14] scan total [15] find_bin bin [16] find_bin before
// [17] find_bin(rev) bin [18] find_bin(rev) before [19..19+nth) exclusive scan per thread
constexpr int kOut = 19;
}  // namespace

extern "C" __global__ void k_blk_test(const int64_t* in, const int32_t* cnt, int64_t kq, int64_t* out, int rounds) {
  extern __shared__ __align__(16) unsigned char smem[];
  GpuBlk B{(int64_t*)smem};
  uint32_t* hist = (uint32_t*)(smem + kRedBytes);
  const int t = B.tid();
  const int64_t v = in[blockIdx.x * B.nth() + t];
  int64_t* o = out + (size_t)blockIdx.x * (kOut + B.nth());
  // Repeat the sequence so that both scratch areas are reused many times.
  for (int r = 0; r < rounds; r++) {
    const int64_t s = B.sum64(v);
    const int64_t mn = B.min64(v);
    const int64_t mx = B.max64(v);
    const uint64_t mu = B.minu64((uint64_t)v);
    const uint64_t an = B.and64((uint64_t)v);
    const uint64_t on = B.or64((uint64_t)v);
    int64_t x = v, y = v ^ 0x5555;
    B.sum2(x, y);
    int64_t m2 = v, s2 = v >> 3;
    B.maxsum(m2, s2);
    const bool an1 = B.any(v == in[blockIdx.x * B.nth()] && t == B.nth() - 1);
    const int64_t bc = B.bcast(v * 3 + r);
    uint64_t a3 = (uint64_t)v, o3 = (uint64_t)v;
    B.andor(a3, o3);
    int32_t tot;
    const int32_t ex = B.excl_scan(cnt[blockIdx.x * B.nth() + t], &tot);
    for (int i = t; i < 256; i += B.nth()) hist[i] = 0;
    B.sync();
    atomicAdd(&hist[(uint64_t)v & 255], 1u);
    int64_t before, before2;
    const int bin = B.find_bin(hist, kq, &before, false);
    const int bin2 = B.find_bin(hist, kq, &before2, true);
    if (r == rounds - 1) {
      if (t == 0) {
        o[0] = s;
        o[1] = mn;
        o[2] = mx;
        o[3] = (int64_t)mu;
        o[4] = (int64_t)an;
        o[5] = (int64_t)on;
        o[6] = x;
        o[7] = y;
        o[8] = m2;
        o[9] = s2;
        o[10] = an1;
        o[11] = bc;
        o[12] = (int64_t)a3;
        o[13] = (int64_t)o3;
        o[14] = tot;
        o[15] = bin;
        o[16] = before;
        o[17] = bin2;
        o[18] = before2;
      }
      o[kOut + t] = ex;
    }
    B.sync();
  }
}

// Returns the number of mismatches (0 = pass); msg gets the first one.
extern "C" int kp_blk_selftest(int nth, int nblocks, uint64_t seed, char* msg, int msg_len) {
  const int n = nth * nblocks;
  std::vector<int64_t> in(n);
  std::vector<int32_t> cnt(n);
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
  auto rnd = [&]() {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return x;
  };
  for (int i = 0; i < n; i++) {
    const uint64_t r = rnd();
    switch (i % 4) {
      case 0: in[i] = (int64_t)r; break;
      case 1: in[i] = (int64_t)(r % 1000) - 500; break;
      case 2: in[i] = (int64_t)(r >> 20); break;
      default: in[i] = -(int64_t)(r >> 3); break;
    }
    cnt[i] = (int32_t)(rnd() % 7);
  }
  const int64_t kq = (int64_t)(rnd() % nth) + 1;
  int64_t *din, *dout;
  int32_t* dcnt;
  const size_t outn = (size_t)nblocks * (kOut + nth);
  if (hipMalloc(&din, 8 * n) || hipMalloc(&dcnt, 4 * n) || hipMalloc(&dout, 8 * outn)) {
    snprintf(msg, msg_len, "hipMalloc failed");
    return -1;
  }
  (void)hipMemcpy(din, in.data(), 8 * n, hipMemcpyHostToDevice);
  (void)hipMemcpy(dcnt, cnt.data(), 4 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_blk_test, dim3(nblocks), dim3(nth), kRedBytes + 1024, 0, din, dcnt, kq, dout, 5);
  if (hipDeviceSynchronize() != hipSuccess) {
    snprintf(msg, msg_len, "kernel failed: %s", hipGetErrorString(hipGetLastError()));
    return -1;
  }
  std::vector<int64_t> out(outn);
  (void)hipMemcpy(out.data(), dout, 8 * outn, hipMemcpyDeviceToHost);
  (void)hipFree(din);
  (void)hipFree(dcnt);
  (void)hipFree(dout);
  int bad = 0;
  auto check = [&](int blk, const char* what, int64_t got, int64_t want) {
    if (got != want) {
      if (!bad) snprintf(msg, msg_len, "nth=%d block %d %s: got %lld want %lld", nth, blk, what, (long long)got,
                         (long long)want);
      bad++;
    }
  };
  for (int b = 0; b < nblocks; b++) {
    const int64_t* v = in.data() + (size_t)b * nth;
    const int32_t* c = cnt.data() + (size_t)b * nth;
    const int64_t* o = out.data() + (size_t)b * (kOut + nth);
    int64_t s = 0, mn = INT64_MAX, mx = INT64_MIN, sy = 0, m2 = INT64_MIN, s2 = 0;
    uint64_t mu = ~0ull, an = ~0ull, on = 0;
    for (int i = 0; i < nth; i++) {
      s += v[i];
      mn = v[i] < mn ? v[i] : mn;
      mx = v[i] > mx ? v[i] : mx;
      mu = (uint64_t)v[i] < mu ? (uint64_t)v[i] : mu;
      an &= (uint64_t)v[i];
      on |= (uint64_t)v[i];
      sy += v[i] ^ 0x5555;
      m2 = v[i] > m2 ? v[i] : m2;
      s2 += v[i] >> 3;
    }
    check(b, "sum64", o[0], s);
    check(b, "min64", o[1], mn);
    check(b, "max64", o[2], mx);
    check(b, "minu64", o[3], (int64_t)mu);
    check(b, "and64", o[4], (int64_t)an);
    check(b, "or64", o[5], (int64_t)on);
    check(b, "sum2.x", o[6], s);
    check(b, "sum2.y", o[7], sy);
    check(b, "maxsum.max", o[8], m2);
    check(b, "maxsum.sum", o[9], s2);
    check(b, "any", o[10], v[nth - 1] == v[0] ? 1 : 0);
    check(b, "bcast", o[11], v[0] * 3 + 4);
    check(b, "andor.and", o[12], (int64_t)an);
    check(b, "andor.or", o[13], (int64_t)on);
    int64_t run = 0;
    for (int i = 0; i < nth; i++) {
      check(b, "excl_scan", o[kOut + i], run);
      run += c[i];
    }
    check(b, "scan total", o[14], run);
    int64_t h[256] = {0};
    for (int i = 0; i < nth; i++) h[(uint64_t)v[i] & 255]++;
    for (int rev = 0; rev < 2; rev++) {
      int64_t acc = 0;
      int bin = rev ? 0 : 255;
      int64_t before = 0;
      for (int q = 0; q < 256; q++) {
        const int idx = rev ? 255 - q : q;
        if (acc + h[idx] >= kq || q == 255) {
          bin = idx;
          before = acc;
          break;
        }
        acc += h[idx];
      }
      check(b, rev ? "find_bin(rev).bin" : "find_bin.bin", o[15 + 2 * rev], bin);
      check(b, rev ? "find_bin(rev).before" : "find_bin.before", o[16 + 2 * rev], before);
    }
  }
  return bad;
}

// ---------------------------------------------------------------------------
// sort.Sort wave emulation (kp_pdq.h) on the device: wave 0 of each block
// sorts its own list in LDS; the host compares with the serial emulation.
// ---------------------------------------------------------------------------
extern "C" __global__ void k_pdq_test(const int32_t* reps, const int32_t* offs, uint32_t* out_names,
                                      int32_t* out_ok) {
  extern __shared__ __align__(16) unsigned char smem[];
  GpuBlk B{(int64_t*)smem};
  const int a = offs[blockIdx.x], n = offs[blockIdx.x + 1] - a;
  PdqWave<GpuBlk> pw = pdq_carve(B, smem + kRedBytes, n);
  for (int i = B.tid(); i < n; i += B.nth()) {
    pw.name[i] = (uint32_t)i;
    pw.rep[i] = reps[a + i];
  }
  B.sync();
  int ok = 1;
  if (B.wid() == 0) ok = pw.run(n) ? 1 : 0;
  ok = B.bcast(ok);
  for (int i = B.tid(); i < n; i += B.nth()) out_names[a + i] = pw.name[i];
  if (B.tid() == 0) out_ok[blockIdx.x] = ok;
}

// Sorts nl lists (concatenated in reps, list j = [offs[j], offs[j+1])) on the
// device; out_names gets each list's permutation (indices into the list).
// Returns the number of lists the wave form declined, or -1 on a HIP error.
extern "C" int kp_pdq_selftest(const int32_t* reps, const int32_t* offs, int nl, int nth, uint32_t* out_names,
                               char* msg, int msg_len) {
  const int total = offs[nl];
  int maxn = 0;
  for (int j = 0; j < nl; j++) maxn = offs[j + 1] - offs[j] > maxn ? offs[j + 1] - offs[j] : maxn;
  int32_t *dr, *doffs, *dok;
  uint32_t* dn;
  if (hipMalloc(&dr, 4 * (size_t)(total + 1)) || hipMalloc(&doffs, 4 * (size_t)(nl + 1)) ||
      hipMalloc(&dn, 4 * (size_t)(total + 1)) || hipMalloc(&dok, 4 * (size_t)nl)) {
    snprintf(msg, msg_len, "hipMalloc failed");
    return -1;
  }
  (void)hipMemcpy(dr, reps, 4 * (size_t)total, hipMemcpyHostToDevice);
  (void)hipMemcpy(doffs, offs, 4 * (size_t)(nl + 1), hipMemcpyHostToDevice);
  const size_t smem = kRedBytes + pdq_wave_bytes(maxn);
  if (smem > 65536) (void)hipFuncSetAttribute((const void*)k_pdq_test, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  hipLaunchKernelGGL(k_pdq_test, dim3(nl), dim3(nth), smem, 0, dr, doffs, dn, dok);
  if (hipDeviceSynchronize() != hipSuccess) {
    snprintf(msg, msg_len, "kernel failed: %s", hipGetErrorString(hipGetLastError()));
    return -1;
  }
  std::vector<int32_t> ok(nl);
  (void)hipMemcpy(out_names, dn, 4 * (size_t)total, hipMemcpyDeviceToHost);
  (void)hipMemcpy(ok.data(), dok, 4 * (size_t)nl, hipMemcpyDeviceToHost);
  (void)hipFree(dr);
  (void)hipFree(doffs);
  (void)hipFree(dn);
  (void)hipFree(dok);
  int declined = 0;
  for (int j = 0; j < nl; j++) declined += ok[j] ? 0 : 1;
  return declined;
}

// ---------------------------------------------------------------------------
// webster_reg (kp_select.h): Webster with one party per lane of one wave, in
// registers (k_select_top's subsets of <= 64 candidates). List j (at most 64 votes,
// party i = cluster rank i) with N[j] seats and the name order desc[j]; the host
// compares the seats with the oracle's AllocateWebsterSeats.
// ---------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(64) k_webster_reg_test(const int64_t* votes, const int32_t* offs,
                                                                    const int32_t* Ns, const int32_t* descs,
                                                                    int32_t* seats, int32_t* ok) {
  extern __shared__ __align__(16) unsigned char smem[];
  WaveBlk B{(int64_t*)smem};
  const int a = offs[blockIdx.x], n = offs[blockIdx.x + 1] - a;
  const int l = B.lane();
  const bool has = l < n;
  const int64_t v = has ? votes[a + l] : 0;
  const int64_t V = B.sum64(v);
  bool okb = false;
  const WebRes w = webster_reg(B, has, (uint32_t)l, v, Ns[blockIdx.x], descs[blockIdx.x] != 0, V, &okb);
  if (has) seats[a + l] = web_seats(w, v, (uint32_t)l);
  if (l == 0) ok[blockIdx.x] = okb ? 1 : 0;
}

// Runs nl lists; seats_out gets every party's seats. Returns the number of lists
// webster_reg declined (its step bound), or -1 on a HIP error.
extern "C" int kp_webster_reg_selftest(const int64_t* votes, const int32_t* offs, const int32_t* Ns,
                                       const int32_t* descs, int nl, int32_t* seats_out, char* msg, int msg_len) {
  const int total = offs[nl];
  int64_t* dv;
  int32_t *doffs, *dN, *dd, *ds, *dok;
  if (hipMalloc(&dv, 8 * (size_t)(total + 1)) || hipMalloc(&doffs, 4 * (size_t)(nl + 1)) ||
      hipMalloc(&dN, 4 * (size_t)nl) || hipMalloc(&dd, 4 * (size_t)nl) || hipMalloc(&ds, 4 * (size_t)(total + 1)) ||
      hipMalloc(&dok, 4 * (size_t)nl)) {
    snprintf(msg, msg_len, "hipMalloc failed");
    return -1;
  }
  (void)hipMemcpy(dv, votes, 8 * (size_t)total, hipMemcpyHostToDevice);
  (void)hipMemcpy(doffs, offs, 4 * (size_t)(nl + 1), hipMemcpyHostToDevice);
  (void)hipMemcpy(dN, Ns, 4 * (size_t)nl, hipMemcpyHostToDevice);
  (void)hipMemcpy(dd, descs, 4 * (size_t)nl, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_webster_reg_test, dim3(nl), dim3(64), 64, 0, dv, doffs, dN, dd, ds, dok);
  if (hipDeviceSynchronize() != hipSuccess) {
    snprintf(msg, msg_len, "kernel failed: %s", hipGetErrorString(hipGetLastError()));
    return -1;
  }
  std::vector<int32_t> ok(nl);
  (void)hipMemcpy(seats_out, ds, 4 * (size_t)total, hipMemcpyDeviceToHost);
  (void)hipMemcpy(ok.data(), dok, 4 * (size_t)nl, hipMemcpyDeviceToHost);
  (void)hipFree(dv);
  (void)hipFree(doffs);
  (void)hipFree(dN);
  (void)hipFree(dd);
  (void)hipFree(ds);
  (void)hipFree(dok);
  int declined = 0;
  for (int j = 0; j < nl; j++) declined += ok[j] ? 0 : 1;
  return declined;
}
