// TEST INFRASTRUCTURE ONLY — CPU oracle.
//
// OCaml standard library `Array.sort` (stdlib/array.ml, unchanged from OCaml 4.x through
// 5.x; the reference requires ocaml >= 4.12, cpr.opam). It is an in-place ternary heap
// sort and NOT stable: elements that compare equal end up in an order fixed by the heap
// operations below. The reference calls it through Compare.first / Compare.at_most_first
// (simulator/lib/compare.ml:44-75), e.g. for Ethereum's uncle selection
// (simulator/protocols/ethereum.ml:269), so the tie order is part of the semantics.
// Restated from the published algorithm: build a max-heap with three children per node
// (maxson / trickledown / trickle), then repeatedly move the root to the end, sift a hole
// down to the bottom (bubble) and insert the displaced element upwards (trickleup).
#pragma once
#include <utility>
#include <vector>

namespace oracle {

// cmp(a, b) < 0  <=>  a sorts before b (OCaml compare convention)
template <class T, class Cmp>
void ocaml_array_sort(std::vector<T>& a, Cmp cmp) {
  const int l = (int)a.size();
  // maxson: index of the largest of up to three sons of i; -1 = no son (Bottom i)
  auto maxson = [&](int len, int i) -> int {
    const int i31 = i + i + i + 1;
    int x = i31;
    if (i31 + 2 < len) {
      if (cmp(a[i31], a[i31 + 1]) < 0) x = i31 + 1;
      if (cmp(a[x], a[i31 + 2]) < 0) x = i31 + 2;
      return x;
    }
    if (i31 + 1 < len && cmp(a[i31], a[i31 + 1]) < 0) return i31 + 1;
    if (i31 < len) return i31;
    return -1;
  };
  // trickle: sift e down from position i
  auto trickle = [&](int len, int i, T e) {
    for (;;) {
      const int j = maxson(len, i);
      if (j < 0) {
        a[i] = e;
        return;
      }
      if (cmp(a[j], e) > 0) {
        a[i] = a[j];
        i = j;
      } else {
        a[i] = e;
        return;
      }
    }
  };
  // bubble: move the hole at i to a leaf, returning the leaf position
  auto bubble = [&](int len, int i) -> int {
    for (;;) {
      const int j = maxson(len, i);
      if (j < 0) return i;
      a[i] = a[j];
      i = j;
    }
  };
  auto trickleup = [&](int i, T e) {
    for (;;) {
      const int father = (i - 1) / 3;
      if (cmp(a[father], e) < 0) {
        a[i] = a[father];
        if (father > 0) {
          i = father;
          continue;
        }
        a[0] = e;
        return;
      }
      a[i] = e;
      return;
    }
  };
  for (int i = (l + 1) / 3 - 1; i >= 0; --i) trickle(l, i, a[i]);
  for (int i = l - 1; i >= 2; --i) {
    T e = a[i];
    a[i] = a[0];
    trickleup(bubble(i, 0), e);
  }
  if (l > 1) std::swap(a[0], a[1]);
}

// Compare.at_most_first (compare.ml:66-75): sort, then the first n (all if fewer)
template <class T, class Cmp>
std::vector<T> ocaml_at_most_first(std::vector<T> a, Cmp cmp, int n) {
  ocaml_array_sort(a, cmp);
  if ((int)a.size() > n) a.resize(n);
  return a;
}

}  // namespace oracle
