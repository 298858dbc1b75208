// npd_nth.hpp -- the list-pruning tie rule of the reference, usable from host and device code.
//
// PolarCode.pruneLists (polar.py:777-791) keeps `torch.topk(-metric, L, 0)` and sorts the indices.
// On the CPU, ATen's topk (TopKImpl.h, k*64 > n) fills a queue of (value, index) pairs in list order
// and runs std::nth_element(queue, queue + k - 1, queue_end, comp) with
// comp(x, y) = (isnan(x) && !isnan(y)) || x > y; the surviving set is queue[0 .. k).  When metrics tie
// across the k-th place, WHICH candidate survives depends on that algorithm's exact swap sequence, so
// this is a statement of libstdc++'s introselect (median-of-3 unguarded partition, heap-select after
// 2*lg(n) rounds, insertion sort of the last <= 3 elements).  The SCL kernel calls it only for list
// groups whose metrics tie across the boundary (otherwise the top-L set is unique and found by rank
// counting).  Pinned against std::nth_element and torch.topk by tests/test_oracle_golden.py.
#pragma once

#ifndef NPD_HD
#if defined(__HIPCC__)
#define NPD_HD __host__ __device__
#else
#define NPD_HD
#endif
#endif

namespace npd {
namespace nth {

struct Q {
    float v;
    int i;
};

NPD_HD inline bool isnan_(float x) { return x != x; }
NPD_HD inline bool comp(const Q& x, const Q& y) { return (isnan_(x.v) && !isnan_(y.v)) || (x.v > y.v); }
NPD_HD inline void swap_(Q* a, Q* b) {
    const Q t = *a;
    *a = *b;
    *b = t;
}

NPD_HD inline void push_heap_(Q* first, int hole, int top, Q value) {
    int parent = (hole - 1) / 2;
    while (hole > top && comp(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

NPD_HD inline void adjust_heap_(Q* first, int hole, int len, Q value) {
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (comp(first[child], first[child - 1])) child--;
        first[hole] = first[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        first[hole] = first[child - 1];
        hole = child - 1;
    }
    push_heap_(first, hole, top, value);
}

NPD_HD inline void make_heap_(Q* first, int len) {
    if (len < 2) return;
    int parent = (len - 2) / 2;
    while (true) {
        adjust_heap_(first, parent, len, first[parent]);
        if (parent == 0) return;
        parent--;
    }
}

NPD_HD inline void heap_select_(Q* first, int middle, int last) {
    make_heap_(first, middle);
    for (int i = middle; i < last; ++i)
        if (comp(first[i], first[0])) {
            const Q value = first[i];
            first[i] = first[0];
            adjust_heap_(first, 0, middle, value);
        }
}

NPD_HD inline void move_median_to_first_(Q* q, int result, int a, int b, int c) {
    if (comp(q[a], q[b])) {
        if (comp(q[b], q[c])) swap_(q + result, q + b);
        else if (comp(q[a], q[c])) swap_(q + result, q + c);
        else swap_(q + result, q + a);
    } else if (comp(q[a], q[c])) {
        swap_(q + result, q + a);
    } else if (comp(q[b], q[c])) {
        swap_(q + result, q + c);
    } else {
        swap_(q + result, q + b);
    }
}

NPD_HD inline int unguarded_partition_(Q* q, int first, int last, int pivot) {
    while (true) {
        while (comp(q[first], q[pivot])) ++first;
        --last;
        while (comp(q[pivot], q[last])) --last;
        if (!(first < last)) return first;
        swap_(q + first, q + last);
        ++first;
    }
}

NPD_HD inline void insertion_sort_(Q* q, int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
        const Q val = q[i];
        if (comp(val, q[first])) {
            for (int j = i; j > first; --j) q[j] = q[j - 1];
            q[first] = val;
        } else {
            int hole = i, next = i - 1;
            while (comp(val, q[next])) {
                q[hole] = q[next];
                hole = next;
                --next;
            }
            q[hole] = val;
        }
    }
}

NPD_HD inline int lg_(int n) {
    int r = 0;
    while (n > 1) {
        n >>= 1;
        ++r;
    }
    return r;
}

// std::nth_element(q, q + nth, q + n, comp)
NPD_HD inline void nth_element(Q* q, int nth, int n) {
    if (n == 0 || nth == n) return;
    int first = 0, last = n;
    int depth = 2 * lg_(n);
    while (last - first > 3) {
        if (depth == 0) {
            heap_select_(q + first, nth + 1 - first, last - first);
            swap_(q + first, q + nth);
            return;
        }
        --depth;
        const int mid = first + (last - first) / 2;
        move_median_to_first_(q, first, first + 1, mid, last - 1);
        const int cut = unguarded_partition_(q, first + 1, last, first);
        if (cut <= nth) first = cut;
        else last = cut;
    }
    insertion_sort_(q, first, last);
}

// Survivor bit mask of pruneLists over n candidates with values v[c] = -metric[c] (list order), keep k.
NPD_HD inline unsigned prune_mask(const float* negm, int n, int k) {
    Q q[16];
    for (int c = 0; c < n; ++c) q[c] = Q{negm[c], c};
    nth_element(q, k - 1, n);
    unsigned m = 0;
    for (int c = 0; c < k; ++c) m |= 1u << q[c].i;
    return m;
}

}  // namespace nth
}  // namespace npd
