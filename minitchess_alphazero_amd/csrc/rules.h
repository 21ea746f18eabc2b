// MinitChess rules on 30-square bitboards, shared by host and device code.
//
// Replaces the python-chess "minitchess" fork the reference consumes through
// exp/environment.py:25-82 (Board(fen), legal_moves, push, result, fen).  The
// rule content is the build's RULES.md (the fork is un-vendored);
// bit-for-bit agreement with oracle/rules.py is tested (tests/test_capi_cpu.py
// on the CPU, tests/test_gpu_rules.py on the GPU).
//
// Geometry: 5 files x 6 ranks, square = 5*rank + file, bit `sq` of
// a uint32_t.  Ray directions: 0 N(+5) 1 S(-5) 2 E(+1) 3 W(-1) 4 NE(+6)
// 5 NW(+4) 6 SE(-4) 7 SW(-6); 0,2,4,5 increase the square index.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HD __host__ __device__ __forceinline__

namespace mtaz {

constexpr int NSQ = 30;
constexpr uint32_t ALL_SQ = (1u << NSQ) - 1;
constexpr int NUM_ACTIONS = 554;

enum PieceType { EMPTY = 0, PAWN = 1, KNIGHT = 2, BISHOP = 3, ROOK = 4, QUEEN = 5, KING = 6 };

// rules_flags bits (RULES.md); the move cap travels separately.
enum RuleFlags : uint32_t {
  RF_DOUBLE_STEP = 1u << 0,
  RF_PROMO_ALL = 1u << 1,
  RF_INSUFFICIENT = 1u << 2,
  RF_FIVEFOLD = 1u << 3,
  RF_SEVENTYFIVE = 1u << 4,
};
constexpr uint32_t RF_DEFAULT = RF_PROMO_ALL | RF_INSUFFICIENT | RF_FIVEFOLD | RF_SEVENTYFIVE;

// Packed position = the MCTS transposition key (exp/agent.py:56 keys nodes by the
// 4-field FEN: board, turn, halfmove, fullmove).  20 bytes:
//   sq[0..3]: 30 nibbles, square s in word s>>3 at bit 4*(s&7); 0 empty,
//             1..6 white P N B R Q K, 9..14 black (8 | type)
//   info:     bit 0 white-to-move, bits 8..15 halfmove clock, bits 16..31 fullmove
struct Pos {
  uint32_t sq[4];
  uint32_t info;
};

// Working form: occupancy per colour + piece-type masks (both colours).
struct BB {
  uint32_t w, b;                        // white / black occupancy
  uint32_t pawn, knight, bishop, rook, queen, king;
  int white;                            // side to move
  int half, full;
};

struct RuleTables {
  uint32_t knight[NSQ], king[NSQ];
  uint32_t pawn_att[2][NSQ];            // [0 white / 1 black][sq]: squares a pawn on sq attacks
  uint32_t ray[8][NSQ];                 // squares strictly beyond sq in direction d
  uint32_t dark;                        // a1 dark: (file + rank) even
};

constexpr RuleTables make_rule_tables() {
  RuleTables t{};
  const int kdx[8] = {1, 1, -1, -1, 2, 2, -2, -2}, kdy[8] = {2, -2, 2, -2, 1, -1, 1, -1};
  const int rdx[8] = {0, 0, 1, -1, 1, -1, 1, -1}, rdy[8] = {1, -1, 0, 0, 1, 1, -1, -1};
  for (int sq = 0; sq < NSQ; ++sq) {
    const int f = sq % 5, r = sq / 5;
    for (int i = 0; i < 8; ++i) {
      int ff = f + kdx[i], rr = r + kdy[i];
      if (ff >= 0 && ff < 5 && rr >= 0 && rr < 6) t.knight[sq] |= 1u << (rr * 5 + ff);
    }
    for (int dx = -1; dx <= 1; ++dx)
      for (int dy = -1; dy <= 1; ++dy) {
        if (!dx && !dy) continue;
        int ff = f + dx, rr = r + dy;
        if (ff >= 0 && ff < 5 && rr >= 0 && rr < 6) t.king[sq] |= 1u << (rr * 5 + ff);
      }
    for (int c = 0; c < 2; ++c) {
      int rr = r + (c == 0 ? 1 : -1);
      for (int dx = -1; dx <= 1; dx += 2) {
        int ff = f + dx;
        if (ff >= 0 && ff < 5 && rr >= 0 && rr < 6) t.pawn_att[c][sq] |= 1u << (rr * 5 + ff);
      }
    }
    for (int d = 0; d < 8; ++d) {
      int ff = f + rdx[d], rr = r + rdy[d];
      while (ff >= 0 && ff < 5 && rr >= 0 && rr < 6) {
        t.ray[d][sq] |= 1u << (rr * 5 + ff);
        ff += rdx[d];
        rr += rdy[d];
      }
    }
    if (((f + r) & 1) == 0) t.dark |= 1u << sq;
  }
  return t;
}

static __constant__ RuleTables d_rules = make_rule_tables();
static constexpr RuleTables h_rules = make_rule_tables();

#if defined(__HIP_DEVICE_COMPILE__)
#define MTAZ_RT d_rules
#else
#define MTAZ_RT h_rules
#endif

HD int lsb(uint32_t x) { return __builtin_ctz(x); }
HD int msb(uint32_t x) { return 31 - __builtin_clz(x); }
HD int popc(uint32_t x) { return __builtin_popcount(x); }

// Every table lookup below goes through `RT`: the constant tables by default; device kernels
// that generate moves pass a copy in LDS (load_rules_lds, mtaz_device.hip).
HD uint32_t slide_pos(int d, int sq, uint32_t occ, const RuleTables& RT = MTAZ_RT) {
  uint32_t a = RT.ray[d][sq];
  uint32_t bl = a & occ;
  if (bl) a &= ~RT.ray[d][lsb(bl)];
  return a;
}
HD uint32_t slide_neg(int d, int sq, uint32_t occ, const RuleTables& RT = MTAZ_RT) {
  uint32_t a = RT.ray[d][sq];
  uint32_t bl = a & occ;
  if (bl) a &= ~RT.ray[d][msb(bl)];
  return a;
}
HD uint32_t rook_att(int sq, uint32_t occ, const RuleTables& RT = MTAZ_RT) {
  return slide_pos(0, sq, occ, RT) | slide_neg(1, sq, occ, RT) | slide_pos(2, sq, occ, RT) | slide_neg(3, sq, occ, RT);
}
HD uint32_t bishop_att(int sq, uint32_t occ, const RuleTables& RT = MTAZ_RT) {
  return slide_pos(4, sq, occ, RT) | slide_pos(5, sq, occ, RT) | slide_neg(6, sq, occ, RT) | slide_neg(7, sq, occ, RT);
}

HD int piece_type_at(const BB& b, int sq) {
  const uint32_t m = 1u << sq;
  if (b.pawn & m) return PAWN;
  if (b.knight & m) return KNIGHT;
  if (b.bishop & m) return BISHOP;
  if (b.rook & m) return ROOK;
  if (b.queen & m) return QUEEN;
  if (b.king & m) return KING;
  return EMPTY;
}

// Is `sq` attacked by side `by_white`?  (oracle/rules.py is_attacked)
HD bool attacked(const BB& b, int sq, int by_white, const RuleTables& RT = MTAZ_RT) {
  const uint32_t x = by_white ? b.w : b.b;
  const uint32_t occ = b.w | b.b;
  if (RT.knight[sq] & b.knight & x) return true;
  if (RT.king[sq] & b.king & x) return true;
  // a pawn of colour X on p attacks sq  <=>  p is attacked from sq by a pawn of the other colour
  if (RT.pawn_att[by_white ? 1 : 0][sq] & b.pawn & x) return true;
  if (rook_att(sq, occ, RT) & (b.rook | b.queen) & x) return true;
  if (bishop_att(sq, occ, RT) & (b.bishop | b.queen) & x) return true;
  return false;
}

HD int king_sq(const BB& b, int white) {
  const uint32_t k = b.king & (white ? b.w : b.b);
  return k ? lsb(k) : -1;
}

HD bool in_check(const BB& b, const RuleTables& RT = MTAZ_RT) {
  const int k = king_sq(b, b.white);
  return k >= 0 && attacked(b, k, !b.white, RT);
}

// Pseudo-legal destinations of the side-to-move piece on sq (oracle pseudo_targets).
HD uint32_t pseudo_targets(const BB& b, int sq, uint32_t flags, const RuleTables& RT = MTAZ_RT) {
  const uint32_t own = b.white ? b.w : b.b, opp = b.white ? b.b : b.w;
  const uint32_t occ = own | opp;
  const int t = piece_type_at(b, sq);
  switch (t) {
    case PAWN: {
      uint32_t out = 0;
      const int fwd = b.white ? sq + 5 : sq - 5;
      if (fwd >= 0 && fwd < NSQ && !((occ >> fwd) & 1u)) {
        out |= 1u << fwd;
        const int start_rank = b.white ? 1 : 4;
        if ((flags & RF_DOUBLE_STEP) && sq / 5 == start_rank) {
          const int f2 = b.white ? fwd + 5 : fwd - 5;
          if (!((occ >> f2) & 1u)) out |= 1u << f2;
        }
      }
      out |= RT.pawn_att[b.white ? 0 : 1][sq] & opp;
      return out;
    }
    case KNIGHT: return RT.knight[sq] & ~own;
    case KING: return RT.king[sq] & ~own;
    case BISHOP: return bishop_att(sq, occ, RT) & ~own;
    case ROOK: return rook_att(sq, occ, RT) & ~own;
    case QUEEN: return (rook_att(sq, occ, RT) | bishop_att(sq, occ, RT)) & ~own;
    default: return 0;
  }
}

HD void clear_sq(BB& b, uint32_t m) {
  const uint32_t k = ~m;
  b.w &= k; b.b &= k; b.pawn &= k; b.knight &= k; b.bishop &= k; b.rook &= k; b.queen &= k; b.king &= k;
}
// selects, not a switch (which the device compiler lowers to an indexed store through scratch)
HD void set_piece(BB& b, int sq, int type, int white) {
  const uint32_t m = 1u << sq;
  b.w |= white ? m : 0u;
  b.b |= white ? 0u : m;
  b.pawn |= type == PAWN ? m : 0u;
  b.knight |= type == KNIGHT ? m : 0u;
  b.bishop |= type == BISHOP ? m : 0u;
  b.rook |= type == ROOK ? m : 0u;
  b.queen |= type == QUEEN ? m : 0u;
  b.king |= type == KING ? m : 0u;
}

// python-chess Board.push for a (from, to, promotion) move of the side to move:
// halfmove reset on captures and pawn moves, fullmove += 1 after black moves.
HD BB make_move(const BB& b, int from, int to, int promo) {
  BB n = b;
  const int t = piece_type_at(b, from);
  const uint32_t opp = b.white ? b.b : b.w;
  const bool zeroing = (t == PAWN) || ((opp >> to) & 1u);
  clear_sq(n, (1u << from) | (1u << to));
  set_piece(n, to, promo ? promo : t, b.white);
  n.half = zeroing ? 0 : b.half + 1;
  if (!b.white) n.full = b.full + 1;
  n.white = !b.white;
  return n;
}

HD bool is_zeroing(const BB& b, int from, int to) {
  const uint32_t opp = b.white ? b.b : b.w;
  return ((b.pawn >> from) & 1u) || ((opp >> to) & 1u);
}

// Legal destinations of the piece on sq: pseudo targets that do not leave the
// mover's king attacked (oracle Board._gen_legal).
HD uint32_t legal_targets(const BB& b, int sq, uint32_t flags, const RuleTables& RT = MTAZ_RT) {
  uint32_t ps = pseudo_targets(b, sq, flags, RT);
  if (!ps) return 0;
  const int ksq0 = king_sq(b, b.white);
  const bool is_king = (b.king >> sq) & 1u;
  uint32_t out = 0;
  while (ps) {
    const int to = lsb(ps);
    ps &= ps - 1;
    BB n = b;
    clear_sq(n, (1u << sq) | (1u << to));
    set_piece(n, to, piece_type_at(b, sq), b.white);
    const int k = is_king ? to : ksq0;
    if (k < 0 || !attacked(n, k, !b.white, RT)) out |= 1u << to;
  }
  return out;
}

// Multiplicity of a legal (from, to) in the reference's legal list: a pawn
// reaching the last rank is listed once per promotion piece (exp/environment.py:48-50
// keeps duplicates of the uci[:4] code).
HD int move_mult(const BB& b, int from, int to, uint32_t flags) {
  if (!((b.pawn >> from) & 1u)) return 1;
  const int last = b.white ? 5 : 0;
  if (to / 5 != last) return 1;
  return (flags & RF_PROMO_ALL) ? 4 : 1;
}

// python-chess has_insufficient_material(color) on the 5x6 board.
HD bool side_insufficient(const BB& b, int white, const RuleTables& RT = MTAZ_RT) {
  const uint32_t own = white ? b.w : b.b, opp = white ? b.b : b.w;
  if (own & (b.pawn | b.rook | b.queen)) return false;
  if (own & b.knight) return popc(own) <= 2 && !(opp & ~b.king & ~b.queen);
  if (own & b.bishop) {
    const uint32_t dark = RT.dark, light = ALL_SQ & ~dark;
    const bool same = !(b.bishop & dark) || !(b.bishop & light);
    return same && !b.pawn && !b.knight;
  }
  return true;
}
HD bool insufficient_material(const BB& b, const RuleTables& RT = MTAZ_RT) {
  return side_insufficient(b, 1, RT) && side_insufficient(b, 0, RT);
}

enum Outcome { ONGOING = 0, DECISIVE = 1, DRAW = 2 };

// Board.result() for a board with no move history (every MCTS episode is
// re-created from a FEN, exp/agent.py:43, so repetition can never trigger there).
// `reps` = number of times the current position occurred (game level only; pass 1).
HD int outcome(const BB& b, int nlegal, bool check, uint32_t flags, int move_cap, int reps,
           const RuleTables& RT = MTAZ_RT) {
  if (nlegal == 0 && check) return DECISIVE;
  if ((flags & RF_SEVENTYFIVE) && b.half >= 150 && nlegal > 0) return DRAW;
  if ((flags & RF_FIVEFOLD) && reps >= 5) return DRAW;
  if ((flags & RF_INSUFFICIENT) && insufficient_material(b, RT)) return DRAW;
  if (nlegal == 0) return DRAW;
  if (move_cap > 0 && b.full > move_cap) return DRAW;
  return ONGOING;
}

// ---- packing ------------------------------------------------------------------------
HD int pos_nib(const Pos& p, int s) { return (p.sq[s >> 3] >> (4 * (s & 7))) & 15; }

// nibble <-> bit-plane transposes: bit i of an 8-bit mask <-> bit 4i of a word
HD uint32_t spread8(uint32_t x) {
  x &= 0xffu;
  x = (x | (x << 12)) & 0x000F000Fu;
  x = (x | (x << 6)) & 0x03030303u;
  return (x | (x << 3)) & 0x11111111u;
}
HD uint32_t gather8(uint32_t x) {
  x &= 0x11111111u;
  x = (x | (x >> 3)) & 0x03030303u;
  x = (x | (x >> 6)) & 0x000F000Fu;
  return (x | (x >> 12)) & 0xffu;
}

// Branch-free through bit planes of the nibbles (type bits 0..2, colour bit 3): a piece type t
// has bit 0 for P B Q (1 3 5), bit 1 for N B K (2 3 6), bit 2 for R Q K (4 5 6).
HD BB unpack(const Pos& p) {
  uint32_t pl[4] = {0, 0, 0, 0};
#pragma unroll
  for (int w = 0; w < 4; ++w)
#pragma unroll
    for (int k = 0; k < 4; ++k) pl[k] |= gather8(p.sq[w] >> k) << (8 * w);
  const uint32_t t0 = pl[0] & ALL_SQ, t1 = pl[1] & ALL_SQ, t2 = pl[2] & ALL_SQ, blk = pl[3] & ALL_SQ;
  BB b{};
  b.pawn = t0 & ~t1 & ~t2;
  b.knight = ~t0 & t1 & ~t2;
  b.bishop = t0 & t1 & ~t2;
  b.rook = ~t0 & ~t1 & t2;
  b.queen = t0 & ~t1 & t2;
  b.king = ~t0 & t1 & t2;
  const uint32_t occ = b.pawn | b.knight | b.bishop | b.rook | b.queen | b.king;
  b.w = occ & ~blk;
  b.b = occ & blk;
  b.white = p.info & 1u;
  b.half = (p.info >> 8) & 0xff;
  b.full = p.info >> 16;
  return b;
}

HD Pos pack(const BB& b) {
  const uint32_t t0 = b.pawn | b.bishop | b.queen, t1 = b.knight | b.bishop | b.king;
  const uint32_t t2 = b.rook | b.queen | b.king, blk = b.b;
  Pos p{};
#pragma unroll
  for (int w = 0; w < 4; ++w)
    p.sq[w] = spread8(t0 >> (8 * w)) | (spread8(t1 >> (8 * w)) << 1) | (spread8(t2 >> (8 * w)) << 2) |
              (spread8(blk >> (8 * w)) << 3);
  const uint32_t half = b.half > 255 ? 255u : (uint32_t)b.half;   // saturates (> the 75-move bound)
  p.info = (b.white ? 1u : 0u) | (half << 8) | ((uint32_t)b.full << 16);
  return p;
}

HD bool pos_eq(const Pos& a, const Pos& c) {
  return a.sq[0] == c.sq[0] && a.sq[1] == c.sq[1] && a.sq[2] == c.sq[2] && a.sq[3] == c.sq[3] && a.info == c.info;
}
// transposition key for repetition: board + turn (python-chess _transposition_key, no clocks)
HD bool pos_eq_board_turn(const Pos& a, const Pos& c) {
  return a.sq[0] == c.sq[0] && a.sq[1] == c.sq[1] && a.sq[2] == c.sq[2] && a.sq[3] == c.sq[3] &&
         ((a.info ^ c.info) & 1u) == 0;
}

HD uint32_t pos_hash(const Pos& p) {
  uint64_t h = 0x9E3779B97F4A7C15ull;
  const uint32_t w[5] = {p.sq[0], p.sq[1], p.sq[2], p.sq[3], p.info};
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    h ^= w[i];
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 32;
  }
  return (uint32_t)h;
}

// ---- encoder (exp/policy.py:82-105) -----------------------------------------------------
// '0prbnqk' token codes indexed by PieceType
HD int token_code(int t) {
  switch (t) {
    case PAWN: return 1;
    case ROOK: return 2;
    case BISHOP: return 3;
    case KNIGHT: return 4;
    case QUEEN: return 5;
    case KING: return 6;
    default: return 0;
  }
}
// tokens[0..29] = side-to-move pieces, tokens[30..59] = opponent pieces, in the
// mover's view: white reads the FEN order (rank 6 first); black the reversed
// string (index 4 + 5*rank - file) with colours swapped.
HD void encode_tokens(const BB& b, uint8_t* tok) {
  const uint32_t own = b.white ? b.w : b.b;
  for (int s = 0; s < NSQ; ++s) {
    const int f = s % 5, r = s / 5;
    const int i = b.white ? (5 - r) * 5 + f : 4 + 5 * r - f;
    const int t = piece_type_at(b, s);
    const int c = token_code(t);
    const bool mine = (own >> s) & 1u;
    tok[i] = mine ? c : 0;
    tok[30 + i] = (t && !mine) ? c : 0;
  }
}
HD float encode_clock(const BB& b) {
  double c = (double)b.full + (b.white ? 0.0 : 0.5);
  return (float)(c / 30.0);
}

}  // namespace mtaz
