// kp_pdq.h — Go sort.Sort (pdqsort) over a TargetClustersList, emulated by ONE
// wave64 with exactly the serial emulation's result (pdqsort_go, kp_algo.h).
//
// Only the O(n) steps are lane-parallel; the control flow (pivot choice,
// breakPatterns, the loop state) is computed redundantly by every lane from the
// same LDS words, so it stays identical to the serial loop. What makes the
// parallel steps exact:
//  - partition / partitionEqual are Hoare scans: the k-th element that stops the
//    left scan is swapped with the k-th element that stops the right scan, for
//    as long as the left one lies before the right one. Both stop lists come
//    from one ballot sweep; the swaps are then independent.
//  - partialInsertionSort's shifts are rotations by one place, found by a
//    ballot search for the stopping element.
//  - the segments the loop recurses into are disjoint, and the only element
//    outside its own segment a step reads is the one before it (a-1), which no
//    later step moves. So pending segments can be processed in any order, and
//    short ones are handed to single lanes (kPdqSerialMax) to run the serial
//    pdqsort_go from the same loop state.
// The shift to the left in partialInsertionSort runs to index 1, not to a
// (sort/zsortinterface.go); it cannot pass a because every element of a segment
// sorts at or after a-1. The wave form checks that instead of assuming it and
// reports failure (caller falls back to the serial sort) if it ever did not.
#pragma once
#include "kp_algo.h"

namespace kp {

struct PdqTask {
  int32_t a, b, limit, st;  // st: bit0 wasBalanced, bit1 wasPartitioned
};
constexpr int kPdqStack = 64;      // pending larger halves (depth <= log2 n + 1)
constexpr int kPdqSerialMax = 24;  // segments this short are sorted by one lane
// LDS bytes: name + rep + stop lists (n each), stack, lane queue.
KP_HD inline size_t pdq_wave_bytes(int n) {
  return 12 * (size_t)((n + 3) & ~3) + sizeof(PdqTask) * (kPdqStack + 64) + 64;
}

template <class BLK>
struct PdqWave {
  const BLK& B;
  uint32_t* name;
  int32_t* rep;
  int32_t* lr;  // stop lists of one partition: left stops ascending | right stops ascending
  PdqTask* stack;
  PdqTask* q;

  KP_FI bool lane0() const { return B.lane() == 0; }
  KP_FI void swap1(int i, int j) const {
    if (lane0()) TCL{name, rep}.Swap(i, j);
    B.wsync();
  }
  // Smallest x in [i, b) with Less(x, x-1), else b.
  KP_FI int first_ascent(int i, int b) const {
    const int W = B.wwidth();
    for (int base = i; base < b; base += W) {
      const int x = base + B.lane();
      const uint64_t m = B.wballot(x < b && rep[x] > rep[x - 1]);
      if (m) return base + ctz64(m);
    }
    return b;
  }
  KP_FI void reverse(int a, int b) const {
    const int W = B.wwidth(), half = (b - a) / 2;
    for (int base = 0; base < half; base += W) {
      const int k = base + B.lane();
      if (k < half) {
        const int i = a + k, j = b - 1 - k;
        const uint32_t ni = name[i], nj = name[j];
        const int32_t ri = rep[i], rj = rep[j];
        name[i] = nj;
        rep[i] = rj;
        name[j] = ni;
        rep[j] = ri;
      }
    }
    B.wsync();
  }
  // Elements [t, p) move one place right (p > t); the element from p goes to t.
  KP_FI void rotate_right(int t, int p) const {
    const int W = B.wwidth();
    const uint32_t en = name[p];
    const int32_t er = rep[p];
    B.wsync();
    for (int hi = p - 1; hi >= t; hi -= W) {
      const int x = hi - B.lane();
      uint32_t vn = 0;
      int32_t vr = 0;
      if (x >= t) {
        vn = name[x];
        vr = rep[x];
      }
      B.wsync();
      if (x >= t) {
        name[x + 1] = vn;
        rep[x + 1] = vr;
      }
      B.wsync();
    }
    if (lane0()) {
      name[t] = en;
      rep[t] = er;
    }
    B.wsync();
  }
  // Elements (p, t] move one place left (t > p); the element from p goes to t.
  KP_FI void rotate_left(int p, int t) const {
    const int W = B.wwidth();
    const uint32_t en = name[p];
    const int32_t er = rep[p];
    B.wsync();
    for (int lo = p + 1; lo <= t; lo += W) {
      const int x = lo + B.lane();
      uint32_t vn = 0;
      int32_t vr = 0;
      if (x <= t) {
        vn = name[x];
        vr = rep[x];
      }
      B.wsync();
      if (x <= t) {
        name[x - 1] = vn;
        rep[x - 1] = vr;
      }
      B.wsync();
    }
    if (lane0()) {
      name[t] = en;
      rep[t] = er;
    }
    B.wsync();
  }
  // partialInsertionSort (maxSteps 5, shortestShifting 50). *ok = false if the
  // left shift would have passed a (never, see the header).
  KP_FI bool partial_insertion(int a, int b, bool* ok) const {
    const int W = B.wwidth();
    int i = a + 1;
    for (int step = 0; step < 5; step++) {
      i = first_ascent(i, b);
      if (i == b) return true;
      if (b - a < 50) return false;
      swap1(i, i - 1);
      if (i - a >= 2) {  // shift the smaller one (now at i-1) to the left
        const int p = i - 1;
        const int32_t er = rep[p];
        int t = -1;
        for (int hi = p - 1; hi >= a && t < 0; hi -= W) {
          const int x = hi - B.lane();
          const uint64_t m = B.wballot(x >= a && rep[x] >= er);
          if (m) t = hi - ctz64(m) + 1;
        }
        if (t < 0) {
          if (a > 0 && !(rep[a - 1] >= er)) {
            *ok = false;
            return false;
          }
          t = a;
        }
        if (t < p) rotate_right(t, p);
      }
      if (b - i >= 2) {  // shift the greater one (at i) to the right
        const int32_t er = rep[i];
        int t = -1;
        for (int lo = i + 1; lo < b && t < 0; lo += W) {
          const int x = lo + B.lane();
          const uint64_t m = B.wballot(x < b && rep[x] <= er);
          if (m) t = lo + ctz64(m) - 1;
        }
        if (t < 0) t = b - 1;
        if (t > i) rotate_left(i, t);
      }
    }
    return false;
  }
  // Hoare partition of [a+1, b) around the pivot moved to a. Returns the number
  // of elements that go left; *swapped = whether any pair was exchanged.
  // eq (partitionEqual): left = !Less(a, x); else (partition): left = Less(x, a).
  KP_FI int hoare(int a, int b, bool eq, bool* swapped) const {
    const int W = B.wwidth();
    const int32_t pv = rep[a];
    const int lo = a + 1, m = b - lo;
    auto goes_left = [&](int x) { return eq ? (pv <= rep[x]) : (rep[x] > pv); };
    int nr = 0;
    for (int base = 0; base < m; base += W) {
      const int k = base + B.lane();
      nr += popc64(B.wballot(k < m && goes_left(lo + k)));
    }
    const int nl = m - nr;
    int cl = 0, cr = 0;
    for (int base = 0; base < m; base += W) {
      const int k = base + B.lane();
      const bool v = k < m;
      const bool g = v && goes_left(lo + k);
      const uint64_t mg = B.wballot(g), ms = B.wballot(v && !g);
      if (g) lr[nl + cr + popc64(mg & B.wlt())] = lo + k;
      else if (v) lr[cl + popc64(ms & B.wlt())] = lo + k;
      cl += popc64(ms);
      cr += popc64(mg);
    }
    B.wsync();
    // pairs k < s: k-th left stop (lr[k]) before the k-th right stop (lr[m-1-k])
    const int pm = nl < nr ? nl : nr;
    int s = 0;
    for (int base = 0; base < pm; base += W) {
      const int k = base + B.lane();
      const uint64_t mk = B.wballot(k < pm && lr[k] < lr[m - 1 - k]);
      const int c = popc64(mk);
      s += c;
      if (c < W) break;  // the predicate is monotone: no later pair qualifies
    }
    for (int base = 0; base < s; base += W) {
      const int k = base + B.lane();
      if (k < s) {
        const int i = lr[k], j = lr[m - 1 - k];
        const uint32_t ni = name[i], nj = name[j];
        const int32_t ri = rep[i], rj = rep[j];
        name[i] = nj;
        rep[i] = rj;
        name[j] = ni;
        rep[j] = ri;
      }
    }
    B.wsync();
    *swapped = s > 0;
    return nr;
  }
  KP_FI void flush(int& qn) const {
    if (B.lane() < qn) {
      const PdqTask t = q[B.lane()];
      pdqsort_go(TCL{name, rep}, t.a, t.b, t.limit, (t.st & 1) != 0, (t.st & 2) != 0);
    }
    B.wsync();
    qn = 0;
  }
  KP_FI void enqueue(int& qn, int a, int b, int limit, int st) const {
    if (b - a <= 1) return;
    if (lane0()) q[qn] = PdqTask{a, b, limit, st};
    B.wsync();
    if (++qn == B.wwidth()) flush(qn);
  }

  // sort.Sort over name/rep[0, n). false: not emulated (stack overflow or a
  // violated invariant); the arrays are then in an unspecified order.
  KP_FI bool run(int n) const {
    if (n <= 1) return true;
    const TCL d{name, rep};
    int sp = 0, qn = 0;
    int a = 0, b = n, limit = bits_len((uint64_t)n), st = 3;
    for (;;) {
      for (;;) {
        const int length = b - a;
        if (length <= kPdqSerialMax || limit == 0) {
          enqueue(qn, a, b, limit, st);
          break;
        }
        bool wb = (st & 1) != 0, wp = (st & 2) != 0;
        if (!wb) {
          if (lane0()) pdq_break_patterns(d, a, b);
          B.wsync();
          limit--;
        }
        int hint;
        int pivot = pdq_choose_pivot(d, a, b, &hint);
        if (hint == 2) {
          reverse(a, b);
          pivot = (b - 1) - (pivot - a);
          hint = 1;
        }
        if (wb && wp && hint == 1) {
          bool ok = true;
          const bool sorted = partial_insertion(a, b, &ok);
          if (!ok) return false;
          if (sorted) break;
        }
        if (a > 0 && !d.Less(a - 1, pivot)) {  // partitionEqual
          swap1(a, pivot);
          bool sw;
          a = a + 1 + hoare(a, b, true, &sw);
          continue;
        }
        swap1(a, pivot);
        bool sw;
        const int mid = a + hoare(a, b, false, &sw);
        swap1(mid, a);
        wp = !sw;
        const int leftLen = mid - a, rightLen = b - mid, thr = length / 8;
        PdqTask large;
        if (leftLen < rightLen) {
          wb = leftLen >= thr;
          large = PdqTask{mid + 1, b, limit, (wb ? 1 : 0) | (wp ? 2 : 0)};
          b = mid;  // the smaller half first, as a fresh recursive call
        } else {
          wb = rightLen >= thr;
          large = PdqTask{a, mid, limit, (wb ? 1 : 0) | (wp ? 2 : 0)};
          a = mid + 1;
        }
        st = 3;
        if (sp == kPdqStack) return false;
        if (lane0()) stack[sp] = large;
        B.wsync();
        sp++;
      }
      if (sp == 0) break;
      sp--;
      const PdqTask t = stack[sp];
      a = t.a;
      b = t.b;
      limit = t.limit;
      st = t.st;
    }
    flush(qn);
    return true;
  }
};

// LDS carve for PdqWave over n elements at p (pdq_wave_bytes(n) bytes).
template <class BLK>
KP_FI PdqWave<BLK> pdq_carve(const BLK& B, unsigned char* p, int n) {
  const int n4 = (n + 3) & ~3;
  uint32_t* name = (uint32_t*)p;
  int32_t* rep = (int32_t*)(name + n4);
  int32_t* lr = rep + n4;
  PdqTask* stack = (PdqTask*)(lr + n4);
  PdqTask* q = stack + kPdqStack;
  return PdqWave<BLK>{B, name, rep, lr, stack, q};
}

}  // namespace kp
