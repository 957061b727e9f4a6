// Go 1.16 sort.Slice on host and device (the Preemptor's sorts: evict.inc on
// the device, the multi-device network verdict in engine.cpp on the host).
#pragma once
#include <hip/hip_runtime.h>

namespace pe {

// Go 1.16 sort.Slice (sort/zsortfunc.go): quickSort_func with doPivot_func's
// ninther and duplicate protection, heapSort_func past the depth limit, and the
// gap-6 shell pass + insertion sort on ranges of <= 12. Not stable: the order
// of equal elements is part of the reference's behaviour. The reference
// recurses into the smaller side and loops on the larger; sub-ranges are
// disjoint and each is sorted by the same deterministic steps whatever the
// order, so an explicit stack (larger side pushed, smaller side continued:
// at most log2(n) pending frames) gives the identical permutation.
template <class Idx, class Less>
struct GoSortDev {
    Idx* d;
    Less less;
    __host__ __device__ __forceinline__ bool L(int i, int j) const { return less(d[i], d[j]); }
    __host__ __device__ __forceinline__ void S(int i, int j) const { const Idx t = d[i]; d[i] = d[j]; d[j] = t; }
    __host__ __device__ void insertion(int a, int b) const {
        for (int i = a + 1; i < b; i++)
            for (int j = i; j > a && L(j, j - 1); j--) S(j, j - 1);
    }
    __host__ __device__ void sift(int lo, int hi, int first) const {
        int root = lo;
        for (;;) {
            int child = 2 * root + 1;
            if (child >= hi) return;
            if (child + 1 < hi && L(first + child, first + child + 1)) child++;
            if (!L(first + root, first + child)) return;
            S(first + root, first + child);
            root = child;
        }
    }
    __host__ __device__ void heap(int a, int b) const {
        const int first = a, hi = b - a;
        for (int i = (hi - 1) / 2; i >= 0; i--) sift(i, hi, first);
        for (int i = hi - 1; i >= 0; i--) { S(first, first + i); sift(0, i, first); }
    }
    __host__ __device__ void median3(int m1, int m0, int m2) const {
        if (L(m1, m0)) S(m1, m0);
        if (L(m2, m1)) { S(m2, m1); if (L(m1, m0)) S(m1, m0); }
    }
    __host__ __device__ void pivot(int lo, int hi, int* midlo, int* midhi) const {
        const int m = (int)((unsigned)(lo + hi) >> 1);
        if (hi - lo > 40) {
            const int s = (hi - lo) / 8;
            median3(lo, lo + s, lo + 2 * s);
            median3(m, m - s, m + s);
            median3(hi - 1, hi - 1 - s, hi - 1 - 2 * s);
        }
        median3(lo, m, hi - 1);
        const int pv = lo;
        int a = lo + 1, c = hi - 1;
        for (; a < c && L(a, pv); a++) {}
        int b = a;
        for (;;) {
            for (; b < c && !L(pv, b); b++) {}
            for (; b < c && L(pv, c - 1); c--) {}
            if (b >= c) break;
            S(b, c - 1);
            b++;
            c--;
        }
        bool protect = hi - c < 5;
        if (!protect && hi - c < (hi - lo) / 4) {
            int dups = 0;
            if (!L(pv, hi - 1)) { S(c, hi - 1); c++; dups++; }
            if (!L(b - 1, pv)) { b--; dups++; }
            if (!L(m, pv)) { S(m, b - 1); b--; dups++; }
            protect = dups > 1;
        }
        if (protect) {
            for (;;) {
                for (; a < b && !L(b - 1, pv); b--) {}
                for (; a < b && L(a, pv); a++) {}
                if (a >= b) break;
                S(a, b - 1);
                a++;
                b--;
            }
        }
        S(pv, b - 1);
        *midlo = b - 1;
        *midhi = c;
    }
    __host__ __device__ void small(int a, int b) const {
        if (b - a > 1) {
            for (int i = a + 6; i < b; i++)
                if (L(i, i - 6)) S(i, i - 6);
            insertion(a, b);
        }
    }
    __host__ __device__ void sort(int n) const {
        if (n <= 12) { small(0, n); return; }   // the common case: no frames
        int depth = 0;
        for (int i = n; i > 0; i >>= 1) depth++;
        int fa[32], fb[32], fd[32];
        int sp = 0;
        fa[0] = 0; fb[0] = n; fd[0] = 2 * depth; sp = 1;
        while (sp > 0) {
            sp--;
            int a = fa[sp], b = fb[sp], dp = fd[sp];
            bool heaped = false;
            while (b - a > 12) {
                if (dp == 0) { heap(a, b); heaped = true; break; }
                dp--;
                int mlo, mhi;
                pivot(a, b, &mlo, &mhi);
                // the reference recurses into [a, mlo) when it is the smaller side
                if (mlo - a < b - mhi) {
                    fa[sp] = mhi; fb[sp] = b; fd[sp] = dp; sp++;   // larger side later
                    b = mlo;
                } else {
                    fa[sp] = a; fb[sp] = mlo; fd[sp] = dp; sp++;
                    a = mhi;
                }
            }
            if (!heaped) small(a, b);
        }
    }
};

template <class Idx, class Less>
__host__ __device__ __forceinline__ void go_sort(Idx* v, int n, Less less) {
    GoSortDev<Idx, Less> g{v, less};
    g.sort(n);
}

}  // namespace pe
