// See java_order.h. Each step names the Java 8 java.util.concurrent.ConcurrentHashMap member it restates.
#include "java_order.h"

#include <charconv>
#include <cmath>
#include <cstring>

#include "plan.h"

namespace sm {

namespace {
constexpr int kTreeify = 8;        // TREEIFY_THRESHOLD
constexpr int kUntreeify = 6;      // UNTREEIFY_THRESHOLD
constexpr int kMinTreeify = 64;    // MIN_TREEIFY_CAPACITY
constexpr int64_t kMaxCap = 1 << 30;  // MAXIMUM_CAPACITY

// spread(h) = (h ^ (h >>> 16)) & HASH_BITS
int32_t spread(int32_t h) { return (int32_t)(((uint32_t)h ^ ((uint32_t)h >> 16)) & 0x7fffffffu); }

// tableSizeFor(c): the power of two >= c
int64_t table_size_for(int64_t c) {
  int64_t n = 1;
  while (n < c && n < kMaxCap) n <<= 1;
  return n;
}
}  // namespace

int32_t java_string_hash(const std::string& s) {
  uint32_t h = 0;
  auto unit = [&](uint32_t u) { h = 31u * h + u; };
  for (size_t i = 0; i < s.size();) {  // UTF-8 → code point → UTF-16 code unit(s)
    const unsigned char c = (unsigned char)s[i];
    uint32_t cp;
    int len;
    if (c < 0x80) { cp = c; len = 1; }
    else if ((c >> 5) == 6) { cp = c & 0x1f; len = 2; }
    else if ((c >> 4) == 14) { cp = c & 0x0f; len = 3; }
    else { cp = c & 0x07; len = 4; }
    for (int k = 1; k < len && i + k < s.size(); ++k) cp = (cp << 6) | ((unsigned char)s[i + k] & 0x3f);
    i += len;
    if (cp >= 0x10000) {
      cp -= 0x10000;
      unit(0xd800 + (cp >> 10));
      unit(0xdc00 + (cp & 0x3ff));
    } else {
      unit(cp);
    }
  }
  return (int32_t)h;
}

namespace {
// Double.toString / Float.toString approximated by the shortest digits that round-trip, laid out as Java does (plain
// decimal for 1e-3 <= |v| < 1e7 with at least one fraction digit, else d.dddE<exp>). Java 8's FloatingDecimal is not
// always shortest, so this is not used for broadcast order: runtime.cpp refuses apps whose broadcasts would order
// float / double keys; it remains for diagnostics only.
template <typename F>
std::string java_fp_string(F v) {
  if (v != v) return "NaN";
  if (std::isinf(v)) return v > 0 ? "Infinity" : "-Infinity";
  if (v == 0) return std::signbit(v) ? "-0.0" : "0.0";
  char b[64];
  auto r = std::to_chars(b, b + sizeof(b), v, std::chars_format::scientific);
  std::string sci(b, r.ptr);  // [-]d[.ddd]e[+-]xx
  std::string out;
  size_t p = 0;
  if (sci[0] == '-') {
    out = "-";
    p = 1;
  }
  const size_t e = sci.find('e');
  std::string digits;
  for (size_t k = p; k < e; ++k)
    if (sci[k] != '.') digits += sci[k];
  const int exp = std::atoi(sci.c_str() + e + 1);
  if (exp >= -3 && exp <= 6) {  // FloatingDecimal: plain when -3 < decExponent < 8 (decExponent = exp + 1)
    if (exp >= 0) {
      std::string ip = digits.substr(0, std::min<size_t>(digits.size(), (size_t)exp + 1));
      while ((int)ip.size() < exp + 1) ip += '0';
      std::string fp = (size_t)exp + 1 < digits.size() ? digits.substr(exp + 1) : "0";
      out += ip + "." + fp;
    } else {
      out += "0." + std::string((size_t)(-exp - 1), '0') + digits;
    }
  } else {
    out += digits.substr(0, 1) + "." + (digits.size() > 1 ? digits.substr(1) : "0") + "E" + std::to_string(exp);
  }
  return out;
}
}  // namespace

std::string java_value_string(int type, int64_t code) {
  switch (type) {
    case T_INT:
    case T_LONG: return std::to_string(code);
    case T_BOOL: return code ? "true" : "false";
    case T_FLOAT: {
      double d;
      memcpy(&d, &code, 8);
      return java_fp_string((float)d);
    }
    case T_DOUBLE: {
      double d;
      memcpy(&d, &code, 8);
      return java_fp_string(d);
    }
    default: return std::to_string(code);
  }
}

// putVal(key, value, false) for an absent key, then addCount(1, binCount)
void JavaChmOrder::put(const std::string& key) {
  const int idx = (int)hash_.size();
  const int32_t h = spread(java_string_hash(key));
  hash_.push_back(h);
  if (tab_.empty()) {  // initTable: DEFAULT_CAPACITY 16, sizeCtl = n - (n >>> 2)
    tab_.resize(16);
    size_ctl_ = 12;
  }
  const size_t i = (size_t)h & (tab_.size() - 1);
  Bin& b = tab_[i];
  int bin_count = 0;
  if (b.nodes.empty()) {
    b.nodes.push_back(idx);  // casTabAt of a new Node into the empty bin
  } else if (!b.tree) {
    bin_count = (int)b.nodes.size();  // nodes walked before pred.next = new Node(...)
    b.nodes.push_back(idx);
  } else {
    bin_count = 2;  // TreeBin.putTreeVal: first = new TreeNode(h, k, v, first, xp)
    b.nodes.insert(b.nodes.begin(), idx);
  }
  if (bin_count >= kTreeify) {  // treeifyBin(tab, i)
    const int64_t n = (int64_t)tab_.size();
    if (n < kMinTreeify) try_presize(n << 1);
    else if (!tab_[i].tree) tab_[i].tree = true;  // new TreeBin(hd): `first` keeps the list order
  }
  // addCount: while (s >= sizeCtl) transfer
  while ((int64_t)hash_.size() >= size_ctl_ && (int64_t)tab_.size() < kMaxCap) transfer();
}

// tryPresize(size)
void JavaChmOrder::try_presize(int64_t size) {
  const int64_t c = size >= (kMaxCap >> 1) ? kMaxCap : table_size_for(size + (size >> 1) + 1);
  for (;;) {
    const int64_t n = (int64_t)tab_.size();
    if (c <= size_ctl_ || n >= kMaxCap) break;
    transfer();
  }
}

// transfer(tab, null), one thread: every bin of the n-table splits into bins i and i + n of the 2n-table
void JavaChmOrder::transfer() {
  const size_t n = tab_.size();
  std::vector<Bin> nt(2 * n);
  for (size_t i = 0; i < n; ++i) {
    const Bin& f = tab_[i];
    if (f.nodes.empty()) continue;
    Bin& ln = nt[i];
    Bin& hn = nt[i + n];
    if (!f.tree) {
      // lastRun: the tail whose nodes all go to the same side keeps its order; the nodes before it are
      // re-linked one by one at the head of their side (ln = new Node(ph, pk, pv, ln))
      const std::vector<int>& L = f.nodes;
      size_t last = 0;
      uint32_t run_bit = (uint32_t)hash_[L[0]] & (uint32_t)n;
      for (size_t k = 1; k < L.size(); ++k) {
        const uint32_t bb = (uint32_t)hash_[L[k]] & (uint32_t)n;
        if (bb != run_bit) {
          run_bit = bb;
          last = k;
        }
      }
      std::vector<int> lo, hi;  // built head-first
      if (run_bit == 0) lo.assign(L.begin() + last, L.end());
      else hi.assign(L.begin() + last, L.end());
      for (size_t k = 0; k < last; ++k) {
        if (((uint32_t)hash_[L[k]] & (uint32_t)n) == 0) lo.insert(lo.begin(), L[k]);
        else hi.insert(hi.begin(), L[k]);
      }
      ln.nodes = std::move(lo);
      hn.nodes = std::move(hi);
    } else {
      // TreeBin: lo / hi lists in `first` order; 6 or fewer nodes untreeify
      for (int x : f.nodes) ((((uint32_t)hash_[x] & (uint32_t)n) == 0) ? ln : hn).nodes.push_back(x);
      ln.tree = (int)ln.nodes.size() > kUntreeify;
      hn.tree = (int)hn.nodes.size() > kUntreeify;
    }
  }
  tab_.swap(nt);
  size_ctl_ = (int64_t)(n << 1) - (int64_t)(n >> 1);
}

// values() iteration (Traverser): bins in index order, each bin's list (a TreeBin: its `first` list)
std::vector<int> JavaChmOrder::order() const {
  std::vector<int> out;
  out.reserve(hash_.size());
  for (const Bin& b : tab_) out.insert(out.end(), b.nodes.begin(), b.nodes.end());
  return out;
}

}  // namespace sm
