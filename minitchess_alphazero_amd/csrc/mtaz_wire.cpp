// Episode wire format: the MQTT payload one puppet publishes per episode.
//
// The reference builds it in Python (app/base.py:63-69):
//   json.dumps({'episode': records, 'userid': ..., 'weights_version': ...,
//               'minitchess_alphazero_version': ...})
// where records are InfoRecorder dicts (exp/callbacks.py:40-54), keys in insertion order
//   observation (FEN), legal_moves (ints), pi (N / N.sum(), float64), action (int), reward (float).
// Here the payloads of a whole batch of games are written straight from the engine's packed
// records (mtaz_records_get), byte-identical to that json.dumps call: CPython's float repr
// (shortest round-trip digits; exponent form when the decimal point position is <= -4 or
// > 16, Python/pystrtod.c format_float_short), json's ensure_ascii string escaping and its
// ", " / ": " separators.  Games are independent, so threads format disjoint game ranges.
#include <algorithm>
#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mtaz.h"

namespace {

// CPython repr(float) (float_repr_style 'short'): the shortest digits that round-trip,
// placed by the rule of format_float_short for mode 'r'.
void put_double(std::string& s, double x) {
  if (std::isnan(x)) { s += "NaN"; return; }            // json.dumps allow_nan=True spellings
  if (std::isinf(x)) { s += x < 0 ? "-Infinity" : "Infinity"; return; }
  char buf[40];
  auto r = std::to_chars(buf, buf + sizeof buf - 1, x, std::chars_format::scientific);
  *r.ptr = 0;                                            // to_chars does not terminate
  // buf = [-]d[.ddd]e(+|-)XX
  const char* p = buf;
  if (*p == '-') { s += '-'; ++p; }
  char dig[24];
  int nd = 0;
  while (*p != 'e') {
    if (*p != '.') dig[nd++] = *p;
    ++p;
  }
  ++p;
  const int e10 = (int)std::strtol(p, nullptr, 10);
  while (nd > 1 && dig[nd - 1] == '0') --nd;            // to_chars never pads, but be safe
  const int decpt = e10 + 1;                             // value = 0.DIGITS x 10^decpt
  if (dig[0] == '0') {                                   // +-0.0
    s += "0.0";
    return;
  }
  if (decpt <= -4 || decpt > 16) {
    s += dig[0];
    if (nd > 1) {
      s += '.';
      s.append(dig + 1, nd - 1);
    }
    char eb[8];
    const int ex = decpt - 1;
    std::snprintf(eb, sizeof eb, "e%c%02d", ex < 0 ? '-' : '+', ex < 0 ? -ex : ex);
    s += eb;
  } else if (decpt <= 0) {
    s += "0.";
    s.append((size_t)(-decpt), '0');
    s.append(dig, nd);
  } else if (decpt >= nd) {
    s.append(dig, nd);
    s.append((size_t)(decpt - nd), '0');
    s += ".0";
  } else {
    s.append(dig, decpt);
    s += '.';
    s.append(dig + decpt, nd - decpt);
  }
}

void put_int(std::string& s, long long v) {
  char b[24];
  auto r = std::to_chars(b, b + sizeof b, v);
  s.append(b, r.ptr);
}

// json.dumps string (ensure_ascii=True): UTF-8 in, \uXXXX (UTF-16 pairs) for non-ASCII.
void put_str(std::string& s, const char* z) {
  if (!z) { s += "null"; return; }
  static const char* HEX = "0123456789abcdef";
  auto u16 = [&](unsigned c) {
    s += "\\u";
    for (int sh = 12; sh >= 0; sh -= 4) s += HEX[(c >> sh) & 15];
  };
  s += '"';
  const unsigned char* p = (const unsigned char*)z;
  while (*p) {
    unsigned c = *p;
    if (c < 0x80) {
      ++p;
      switch (c) {
        case '"': s += "\\\""; break;
        case '\\': s += "\\\\"; break;
        case '\n': s += "\\n"; break;
        case '\r': s += "\\r"; break;
        case '\t': s += "\\t"; break;
        case '\b': s += "\\b"; break;
        case '\f': s += "\\f"; break;
        default:
          if (c < 0x20) u16(c);
          else s += (char)c;
      }
      continue;
    }
    int n = c >= 0xF0 ? 3 : c >= 0xE0 ? 2 : 1;
    unsigned cp = c & (n == 3 ? 0x07 : n == 2 ? 0x0F : 0x1F);
    ++p;
    for (int i = 0; i < n && (*p & 0xC0) == 0x80; ++i, ++p) cp = (cp << 6) | (*p & 0x3F);
    if (cp >= 0x10000) {
      cp -= 0x10000;
      u16(0xD800 | (cp >> 10));
      u16(0xDC00 | (cp & 0x3FF));
    } else {
      u16(cp);
    }
  }
  s += '"';
}

struct Records {
  const int32_t* plies;
  const uint32_t* pos;
  const int32_t* action;
  const int32_t* k;
  const uint16_t* codes;
  const uint32_t* visits;
  const float* reward;
};

void put_episode(std::string& s, const Records& R, int64_t p0, int64_t e0, int plies, const std::string& tail) {
  char fen[96];
  s += "{\"episode\": [";
  int64_t e = e0;
  for (int i = 0; i < plies; ++i) {
    const int64_t p = p0 + i;
    const int k = R.k[p];
    if (i) s += ", ";
    s += "{\"observation\": ";
    mtaz_pos_to_fen(R.pos + 5 * p, fen, sizeof fen);
    put_str(s, fen);
    s += ", \"legal_moves\": [";
    for (int j = 0; j < k; ++j) {
      if (j) s += ", ";
      put_int(s, R.codes[e + j]);
    }
    s += "], \"pi\": [";
    uint64_t sum = 0;
    for (int j = 0; j < k; ++j) sum += R.visits[e + j];  // N.sum(): exact for integer counts
    for (int j = 0; j < k; ++j) {
      if (j) s += ", ";
      put_double(s, (double)R.visits[e + j] / (double)sum);
    }
    s += "], \"action\": ";
    put_int(s, R.action[p]);
    s += ", \"reward\": ";
    put_double(s, (double)R.reward[p]);
    s += '}';
    e += k;
  }
  s += "]";
  s += tail;
}

}  // namespace

extern "C" int mtaz_repr_double(double x, char* buf, int cap) {
  std::string s;
  put_double(s, x);
  if ((int)s.size() + 1 > cap) return MTAZ_E_CAPACITY;
  memcpy(buf, s.c_str(), s.size() + 1);
  return (int)s.size();
}

extern "C" int64_t mtaz_records_json(int n_games, const int32_t* plies, const uint32_t* pos, const int32_t* action,
                                     const int32_t* k, const uint16_t* codes, const uint32_t* visits,
                                     const float* reward, const char* userid, const char* weights_version,
                                     const char* version, char* out, int64_t cap, int64_t* offsets) {
  if (n_games < 0) return MTAZ_E_FAIL;
  const Records R{plies, pos, action, k, codes, visits, reward};
  std::string tail = ", \"userid\": ";
  put_str(tail, userid);
  tail += ", \"weights_version\": ";
  put_str(tail, weights_version);
  tail += ", \"minitchess_alphazero_version\": ";
  put_str(tail, version);
  tail += '}';
  // per-game starts in the ply and entry arrays
  std::vector<int64_t> p0(n_games + 1, 0), e0(n_games + 1, 0);
  for (int g = 0; g < n_games; ++g) {
    p0[g + 1] = p0[g] + plies[g];
    int64_t e = 0;
    for (int i = 0; i < plies[g]; ++i) e += k[p0[g] + i];
    e0[g + 1] = e0[g] + e;
  }
  unsigned hw = std::thread::hardware_concurrency();
  const int T = std::max(1, std::min<int>({16, (int)(hw ? hw : 1), (n_games + 63) / 64}));
  std::vector<std::string> part(T);
  std::vector<std::vector<int64_t>> lens(T);
  auto work = [&](int t) {
    const int g0 = (int)((int64_t)n_games * t / T), g1 = (int)((int64_t)n_games * (t + 1) / T);
    std::string& s = part[t];
    for (int g = g0; g < g1; ++g) {
      const size_t before = s.size();
      put_episode(s, R, p0[g], e0[g], plies[g], tail);
      lens[t].push_back((int64_t)(s.size() - before));
    }
  };
  if (T == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  int64_t total = 0;
  for (auto& s : part) total += (int64_t)s.size();
  if (offsets) offsets[n_games] = total;
  if (!out || total > cap) return total;                  // size query / too small: nothing written
  int64_t o = 0;
  int g = 0;
  for (int t = 0; t < T; ++t) {
    memcpy(out + o, part[t].data(), part[t].size());
    for (int64_t L : lens[t]) {
      if (offsets) offsets[g] = o;
      o += L;
      ++g;
    }
  }
  return total;
}
