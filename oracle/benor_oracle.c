/*
 * benor_oracle.c -- CPU restatement of the reference Ben-Or round loop.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or as the timed CPU baseline).  The product path (libbenor.so) never links
 * or calls anything in oracle/.
 *
 * Reference: viviendbk/ben-or-consensus-algorithm (TypeScript, Express).  The
 * reference cannot be executed in this image (Node 12 has no global fetch and
 * no optional chaining; express / ts-node / jest are absent, no network), so
 * this file restates its algorithm in C.  Parity of this restatement is
 * pinned by the reference's own known-answer tests
 * (__test__/tests/benorconsensus.test.ts:133-486, fixtures in
 * tests/golden/reference_cases.json) and by the exact analytic law of SURVEY
 * §8c (oracle/analytic.py).
 *
 * Two restatements that cross-check each other:
 *   (i)  oracle_message_sim  -- message-level: per-node inbox arrays keyed by
 *        round, literal `>= N-F` triggers, seeded delivery order
 *        (src/nodes/node.ts:43-163, :167-188, :191-194).
 *   (ii) oracle_run_trials   -- round-level bit planes + popcount, the same
 *        semantics the HIP kernel implements; also the timed CPU baseline.
 *
 * Shared conventions (identical in the HIP kernel):
 *   Philox4x32-10, key = {seed_lo, seed_hi}.
 *   coin of the c-th live node (ascending node id) in round r >= 1 =
 *       bit (c & 31) of word (r-1) & 3 of philox(ctr {trial_lo, trial_hi,
 *       c >> 5, ((r-1) >> 2) | 0<<24}): one block per 32 nodes and 4 rounds;
 *       x = coin, the reference's `Math.random() > 0.5 ? 0 : 1` (node.ts:111)
 *       with P(1) = 1/2.
 *   random initial value of the c-th live node (ascending node id), m live
 *       nodes:
 *       m <= 32 (one word per trial, r05): bit c of word trial & 3 of
 *       philox(ctr {q_lo, q_hi, 1<<31, 1<<24}), q = trial >> 2 -- four
 *       consecutive trials share one block;
 *       m > 32: bit (c & 31) of word c>>5, word j = philox(ctr {trial_lo,
 *       trial_hi, j>>2, 1<<24})[j & 3].
 *   halting: the network stops after the round in which every live node has
 *       decided (the reference's all-decided auto-stop, node.ts:116-145,
 *       without its F>0 `decided:null` defect), else after k_max rounds.
 *       A live node's k is then (rounds run) + 1 (node.ts:147).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_STREAM_COIN 0u
#define ORC_STREAM_INIT 1u
#define ORC_STREAM_DELIVERY 2u
#define ORC_STREAM_ORDER 3u

/* ---------------------------------------------------------------- Philox */
/* Philox4x32-10 (Salmon et al., SC'11; Random123 reference constants). */
static inline void orc_mulhilo(uint32_t a, uint32_t b, uint32_t *hi, uint32_t *lo) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    *hi = (uint32_t)(p >> 32);
    *lo = (uint32_t)p;
}

void oracle_philox4x32_10(const uint32_t key_in[2], const uint32_t ctr_in[4], uint32_t out[4]) {
    uint32_t k0 = key_in[0], k1 = key_in[1];
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, lo0, hi1, lo1;
        orc_mulhilo(0xD2511F53u, c0, &hi0, &lo0);
        orc_mulhilo(0xCD9E8D57u, c2, &hi1, &lo1);
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static inline uint32_t orc_philox_word(uint64_t seed, uint64_t trial, uint32_t c2, uint32_t c3, int idx) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)trial, (uint32_t)(trial >> 32), c2, c3};
    uint32_t out[4];
    oracle_philox4x32_10(key, ctr, out);
    return out[idx];
}

/* node.ts:111  `Math.random() > 0.5 ? 0 : 1`: the coin of the c-th live node
 * (compact index) in round r >= 1. */
int oracle_coin(uint64_t seed, uint64_t trial, uint32_t c, uint32_t round) {
    const uint32_t rr = round - 1u;
    uint32_t w = orc_philox_word(seed, trial, c >> 5, ((rr >> 2) & 0x00FFFFFFu) | (ORC_STREAM_COIN << 24),
                                 (int)(rr & 3u));
    return (int)((w >> (c & 31u)) & 1u);
}

/* Random initial value (0/1) of the c-th live node of a network of m live
 * nodes.  A network of at most 32 live nodes needs one 32-bit word per trial,
 * so four consecutive trials share a Philox block (ctr[2] bit 31 marks the
 * shared form); larger networks take words c >> 5 of their own blocks. */
int oracle_random_init(uint64_t seed, uint64_t trial, uint32_t c, uint32_t m) {
    if (m <= 32u) {
        uint32_t w = orc_philox_word(seed, trial >> 2, 1u << 31, ORC_STREAM_INIT << 24, (int)(trial & 3u));
        return (int)((w >> c) & 1u);
    }
    uint32_t j = c >> 5;
    uint32_t w = orc_philox_word(seed, trial, j >> 2, ORC_STREAM_INIT << 24, (int)(j & 3));
    return (int)((w >> (c & 31)) & 1u);
}

/* ---------------------------------------------------- launch validation */
/* launchNodes.ts:10-13.  Returns 0 ok, 1 "Arrays don't match",
 * 2 "faultyList doesnt have F faulties". */
int oracle_validate(int64_t N, int64_t F, int64_t n_init, int64_t n_faulty, const uint8_t *faulty) {
    if (n_init != n_faulty || N != n_init) return 1;
    int64_t cnt = 0;
    for (int64_t i = 0; i < n_faulty; ++i) cnt += faulty[i] ? 1 : 0;
    if (cnt != F) return 2;
    return 0;
}

/* ------------------------------------------------------------ node state */
/* NodeState (src/types.ts:1-8): x -1=null,0,1,2='?'; decided -1=null,0,1; k -1=null */
typedef struct {
    int8_t killed;
    int8_t x;
    int8_t decided;
    int8_t pad;
    int32_t k;
} orc_node_state;

/* ===================================================================== */
/* (i) message-level restatement of node.ts:43-163                        */
/* ===================================================================== */
typedef struct { int32_t k; int8_t x; uint8_t phase; uint32_t to; } orc_msg;   /* {k, x, messageType} */
typedef struct { int8_t *v; int32_t len, cap; } orc_vec;                       /* Value[] */

static void vec_push(orc_vec *a, int8_t x) {
    if (a->len == a->cap) {
        a->cap = a->cap ? a->cap * 2 : 8;
        a->v = (int8_t *)realloc(a->v, (size_t)a->cap);
    }
    a->v[a->len++] = x;
}

typedef struct { uint64_t s; } orc_rng;
static inline uint64_t orc_splitmix(orc_rng *r) {
    uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/*
 * One network run at message granularity.
 *   init[i] in {0,1,2('?')}, faulty[i] in {0,1}; state_out[N].
 *   order_mode 0: FIFO delivery; k >= 1: seeded uniformly random pick from
 *   the pending pool (the "fixed seeded order" of the north star), k salts
 *   the order stream.
 * Returns rounds run R (>=0), or -1 if every live node decided is never
 * reached within k_max (state then reflects k_max rounds).  *stalled is set
 * when the pool drained without a halt (fewer than N-F live senders).
 */
int oracle_message_sim(uint32_t N, uint32_t F, const int8_t *init, const uint8_t *faulty,
                       uint64_t seed, uint64_t trial, uint32_t k_max, int order_mode,
                       orc_node_state *state_out, int *stalled) {
    /* node.ts:21-26 */
    orc_node_state *st = state_out;
    uint32_t live = 0;
    for (uint32_t i = 0; i < N; ++i) {
        st[i].killed = faulty[i] ? 1 : 0;
        st[i].x = faulty[i] ? -1 : init[i];
        st[i].decided = faulty[i] ? -1 : 0;
        st[i].k = faulty[i] ? -1 : 0;
        st[i].pad = 0;
        live += faulty[i] ? 0 : 1;
    }
    if (stalled) *stalled = 0;
    uint32_t *cidx = (uint32_t *)malloc(sizeof(uint32_t) * (N + 1));   /* compact live index (coins) */
    for (uint32_t i = 0, c = 0; i < N; ++i) { cidx[i] = c; c += faulty[i] ? 0 : 1; }
    const int64_t quorum = (int64_t)N - (int64_t)F;
    const uint32_t KR = k_max + 2;
    /* proposals / votes: Map<k, Value[]> per node (node.ts:29-30) */
    orc_vec *prop = (orc_vec *)calloc((size_t)N * KR, sizeof(orc_vec));
    orc_vec *vote = (orc_vec *)calloc((size_t)N * KR, sizeof(orc_vec));
    uint8_t *pdone = (uint8_t *)calloc((size_t)N * KR, 1);   /* first P trigger seen */
    uint32_t *completed = (uint32_t *)calloc(KR, sizeof(uint32_t));

    size_t pcap = (size_t)N * N * 2 + 16, plen = 0;
    orc_msg *pool = (orc_msg *)malloc(pcap * sizeof(orc_msg));
    orc_rng rng;
    rng.s = ((uint64_t)orc_philox_word(seed, trial, 0, ORC_STREAM_ORDER << 24, 0) << 32) |
            orc_philox_word(seed, trial, 0, ORC_STREAM_ORDER << 24, 1);
    rng.s ^= (uint64_t)order_mode * 0xD1B54A32D192ED03ull;   /* order_mode >= 1 salts the order */

#define BCAST(KK, XX, PH)                                                        \
    do {                                                                         \
        for (uint32_t to_ = 0; to_ < N; ++to_) {                                 \
            if (plen == pcap) { pcap *= 2; pool = (orc_msg *)realloc(pool, pcap * sizeof(orc_msg)); } \
            pool[plen].k = (KK); pool[plen].x = (XX); pool[plen].phase = (PH);   \
            pool[plen].to = to_; ++plen;                                         \
        }                                                                        \
    } while (0)

    /* /start (node.ts:167-188), called for every node by startConsensus */
    for (uint32_t i = 0; i < N; ++i) {
        if (!st[i].killed) {
            st[i].k = 1;
            BCAST(1, st[i].x, 0);
        }
    }
    int rounds = 0, halted = 0;
    size_t head = 0;
    while (!halted && head < plen) {
        size_t pick;
        if (order_mode >= 1) {
            size_t avail = plen - head;
            pick = head + (size_t)(orc_splitmix(&rng) % avail);
            orc_msg t = pool[pick]; pool[pick] = pool[head]; pool[head] = t;
        }
        pick = head++;
        orc_msg m = pool[pick];
        uint32_t i = m.to;
        if (st[i].killed) continue;                         /* node.ts:45 */
        if (m.k < 0 || (uint32_t)m.k >= KR) continue;
        if (m.phase == 0) {                                 /* "proposal phase" node.ts:46-82 */
            orc_vec *a = &prop[(size_t)i * KR + (uint32_t)m.k];
            vec_push(a, m.x);
            if ((int64_t)a->len >= quorum) {
                int c0 = 0, c1 = 0;
                for (int32_t j = 0; j < a->len; ++j) {
                    if (a->v[j] == 0) c0++;
                    else if (a->v[j] == 1) c1++;
                }
                int8_t v = (c0 > c1) ? 0 : (c1 > c0) ? 1 : 2;
                BCAST(m.k, v, 1);                           /* node.ts:72-80 */
            }
        } else {                                            /* "voting phase" node.ts:83-158 */
            orc_vec *a = &vote[(size_t)i * KR + (uint32_t)m.k];
            vec_push(a, m.x);
            if ((int64_t)a->len >= quorum) {
                int c0 = 0, c1 = 0;
                for (int32_t j = 0; j < a->len; ++j) {
                    if (a->v[j] == 0) c0++;
                    else if (a->v[j] == 1) c1++;
                }
                if (c0 > (int)F) { st[i].x = 0; st[i].decided = 1; }
                else if (c1 > (int)F) { st[i].x = 1; st[i].decided = 1; }
                else {
                    if (c0 + c1 > 0 && c0 > c1) st[i].x = 0;
                    else if (c0 + c1 > 0 && c0 < c1) st[i].x = 1;
                    else st[i].x = (int8_t)oracle_coin(seed, trial, cidx[i], (uint32_t)m.k);
                }
                st[i].k = m.k + 1;                          /* node.ts:147 */
                uint8_t *pd = &pdone[(size_t)i * KR + (uint32_t)m.k];
                int first = !*pd;
                *pd = 1;
                /* halting rule (all-decided auto-stop, node.ts:116-145): once
                 * every live node has completed round k, stop if all decided
                 * or k == k_max. */
                if (first) {
                    completed[m.k]++;
                    if (completed[m.k] == live) {
                        int all = 1;
                        for (uint32_t j = 0; j < N; ++j)
                            if (!faulty[j] && st[j].decided != 1) { all = 0; break; }
                        rounds = m.k;
                        if (all || (uint32_t)m.k >= k_max) { halted = all ? 2 : 1; break; }
                    }
                }
                BCAST(m.k + 1, st[i].x, 0);                 /* node.ts:149-157 */
            }
        }
    }
#undef BCAST
    if (!halted && stalled) *stalled = 1;
    for (size_t j = 0; j < (size_t)N * KR; ++j) { free(prop[j].v); free(vote[j].v); }
    free(prop); free(vote); free(pdone); free(completed); free(pool); free(cidx);
    if (halted == 2) return rounds;
    return -1;
}

/* ===================================================================== */
/* (ii) round-level bit-plane restatement (same semantics as the kernel)  */
/* ===================================================================== */
typedef struct {
    uint32_t N, F;            /* network size, fault parameter (quorum N-F, decide > F) */
    uint32_t k_max;           /* round cap (>= 1) */
    uint32_t init_mode;       /* 0 = random Bernoulli(1/2) per live node, 1 = fixed */
    uint64_t seed;
    uint64_t trial_begin;
    uint64_t trial_count;
    const uint8_t *faulty;    /* [N] crash-faulty (never send, never receive) */
    const int8_t *init;       /* [N] 0/1/2('?'), used when init_mode == 1 */
    int32_t threads;          /* <=0: all available */
    uint32_t mode;            /* 0 = lockstep (exactly F crashed), 1 = random delivery (f <= F) */
} orc_trials_cfg;

/* ------------------------------------------------ random delivery model */
/* Generalised delivery (no reference counterpart: the
 * reference admits only f == F, launchNodes.ts:12-13).  With f <= F crashed,
 * each live receiver tallies, in each phase, the first N-F arrivals: a
 * uniformly random subset of exactly q = N-F of the m = N-f live senders,
 * independent per (receiver, round, phase).  At f == F it is every live
 * sender, i.e. lockstep.
 *
 * Random words: Philox stream 2, ctr {trial_lo, trial_hi, block |
 * (round & 0x7FFF) << 16 | phase << 31, node | (2 << 24)}, consumed in order
 * (word i = block i>>2, lane i&3).  `node` is the receiver's node id.  Only
 * the last counter word differs between the receivers of a trial, so the
 * GPU computes the first rounds' products that depend only on the other
 * three once per (trial, round, phase, block) (r04, benor_random.hip).
 * Two exact samplers, picked by the plan constants (m, q); k = min(e, q),
 * e = m - q:
 *
 * (a) k < 64 or k * 8 <= m: Floyd's algorithm draws a uniform k-subset T of [0, m): for
 *     j = m-k .. m-1, t = uniform[0, j] (Lemire's multiply-shift with exact
 *     rejection), T += (t in T) ? j : t.  Delivered set = T if q <= e, else
 *     the live senders minus T.
 * (b) otherwise, Bernoulli mask + exact fix-up.  Every sender is included
 *     independently with p = a/16, a = ceil(16 q / m) in [1, 15]: bit = (u < a)
 *     for a 4-bit u whose bit i comes from stream word i of the mask word,
 *     evaluated from bit tz(a) upward as r = a_i ? (~w | r) : (~w & r) (the
 *     bits of u below tz(a) cannot change the comparison and are not drawn),
 *     so each 32-sender mask word takes 4 - tz(a) stream words; bits >= m are
 *     cleared.  Given its count c the mask is a uniform c-subset; then, while
 *     c != q, the next b-bit field (b = ceil(log2 m); floor(32/b) fields per
 *     stream word, low bits first, starting at the Philox block after the
 *     mask's last word) is a sender index idx, and when
 *     idx < m and its bit is set (c > q) or clear (c < q) the bit is flipped:
 *     each flip removes a uniform member (adds a uniform non-member), so the
 *     result is a uniform q-subset.  Cost ~ m/32 words + |c - q| draws instead
 *     of k draws. */
typedef struct {
    uint32_t key[2], ctr[4];
    uint32_t buf[4];
    uint32_t widx;
    uint32_t blk_shift;       /* the block index goes to ctr[2] << blk_shift */
} orc_dstream;

static inline uint32_t dstream_next(orc_dstream *s) {
    if ((s->widx & 3u) == 0) {
        uint32_t c[4] = {s->ctr[0], s->ctr[1], s->ctr[2] | ((s->widx >> 2) << s->blk_shift), s->ctr[3]};
        oracle_philox4x32_10(s->key, c, s->buf);
    }
    return s->buf[s->widx++ & 3u];
}

/* uniform integer in [0, range) (Lemire 2019, exact) */
static inline uint32_t dstream_uniform(orc_dstream *s, uint32_t range) {
    uint64_t m = (uint64_t)dstream_next(s) * range;
    uint32_t l = (uint32_t)m;
    if (l < range) {
        uint32_t t = (uint32_t)(-range) % range;
        while (l < t) {
            m = (uint64_t)dstream_next(s) * range;
            l = (uint32_t)m;
        }
    }
    return (uint32_t)(m >> 32);
}

/* Sampler (b) parameters: p = a/16 and the index field width b. */
int oracle_delivery_bernoulli(uint32_t m, uint32_t q, uint32_t *a_out, uint32_t *b_out) {
    const uint32_t e = m - q, k = q <= e ? q : e;
    if (k < 64u || (uint64_t)k * 8u <= m) return 0;
    uint32_t a = (16u * q + m - 1u) / m;
    if (a < 1u) a = 1u;
    if (a > 15u) a = 15u;
    uint32_t b = 1;
    while ((1u << b) < m) ++b;
    if (a_out) *a_out = a;
    if (b_out) *b_out = b;
    return 1;
}

/* D[W]: delivered-sender mask (compact sender indices) of receiver `node`. */
void oracle_delivery_mask(uint64_t seed, uint64_t trial, uint32_t node, uint32_t round, uint32_t phase,
                          uint32_t m, uint32_t q, uint64_t *D) {
    const uint32_t W = (m + 63) / 64;
    orc_dstream s;
    s.key[0] = (uint32_t)seed; s.key[1] = (uint32_t)(seed >> 32);
    s.ctr[0] = (uint32_t)trial; s.ctr[1] = (uint32_t)(trial >> 32);
    s.ctr[2] = ((round & 0x7FFFu) << 16) | ((phase & 1u) << 31);
    s.ctr[3] = (node & 0xFFFu) | (ORC_STREAM_DELIVERY << 24);
    s.widx = 0;
    s.blk_shift = 0;
    uint32_t a, b;
    if (oracle_delivery_bernoulli(m, q, &a, &b)) {          /* sampler (b) */
        uint32_t M32[128];
        const uint32_t W32 = (m + 31) / 32;
        uint32_t tz = 0;
        while (!((a >> tz) & 1u)) ++tz;
        int64_t c = 0;
        for (uint32_t w = 0; w < W32; ++w) {
            uint32_t r = 0;
            for (uint32_t i = tz; i < 4; ++i) {
                const uint32_t u = dstream_next(&s);
                r = ((a >> i) & 1u) ? (~u | r) : (~u & r);
            }
            const uint32_t n = m - 32u * w;
            if (n < 32u) r &= (1u << n) - 1u;
            M32[w] = r;
            c += __builtin_popcount(r);
        }
        const uint32_t per = 32u / b, fmask = (1u << b) - 1u;
        s.widx = (s.widx + 3u) & ~3u;                       /* fix-up fields start at a fresh block */
        uint32_t word = 0, left = 0;
        while (c != (int64_t)q) {
            if (left == 0) { word = dstream_next(&s); left = per; }
            const uint32_t idx = word & fmask;
            word >>= b;
            --left;
            if (idx >= m) continue;
            const uint32_t bit = (M32[idx >> 5] >> (idx & 31u)) & 1u;
            if (bit == (c > (int64_t)q ? 1u : 0u)) {
                M32[idx >> 5] ^= 1u << (idx & 31u);
                c += bit ? -1 : 1;
            }
        }
        for (uint32_t w = 0; w < W; ++w)
            D[w] = (uint64_t)M32[2 * w] | ((2 * w + 1 < W32) ? (uint64_t)M32[2 * w + 1] << 32 : 0ull);
        return;
    }
    const uint32_t e = m - q;
    const int deliver_T = q <= e;
    const uint32_t k = deliver_T ? q : e;
    uint64_t T[64];
    for (uint32_t w = 0; w < W; ++w) T[w] = 0;
    for (uint32_t j = m - k; j < m; ++j) {
        const uint32_t t = dstream_uniform(&s, j + 1u);
        const uint32_t idx = ((T[t >> 6] >> (t & 63)) & 1ull) ? j : t;
        T[idx >> 6] |= 1ull << (idx & 63);
    }
    for (uint32_t w = 0; w < W; ++w) {
        const uint32_t lo = w * 64, n = (m - lo) < 64 ? (m - lo) : 64;
        const uint64_t vm = n == 64 ? ~0ull : ((1ull << n) - 1);
        D[w] = deliver_T ? T[w] : (vm & ~T[w]);
    }
}

static inline int popc64(uint64_t v) { return __builtin_popcountll(v); }

/* Histogram layout (shared with the kernel):
 *   hist[(R * 3) + v], R in [1, k_max]: all live decided after round R, common x = v (2 = differ)
 *   hist[0 * 3 + v]: not all decided after k_max rounds; v = common x or 2
 *   hist[(k_max + 1) * 3]: count of trials where all decided but values differ */
static void run_one(const orc_trials_cfg *cfg, const uint32_t *live_ids, uint32_t m,
                    uint64_t trial, uint64_t *x0, uint64_t *x1, uint64_t *p0, uint64_t *p1,
                    uint64_t *dec, uint64_t *hist, orc_node_state *node_out) {
    const uint32_t W = (m + 63) / 64;
    const uint32_t F = cfg->F;
    const int64_t quorum = (int64_t)cfg->N - (int64_t)cfg->F;
    const size_t H = (size_t)(cfg->k_max + 1) * 3;
    if (m == 0) { hist[2]++; return; }
    /* initial planes (compact live order) */
    for (uint32_t w = 0; w < W; ++w) { x0[w] = x1[w] = 0; dec[w] = 0; }
    for (uint32_t c = 0; c < m; ++c) {
        int v = cfg->init_mode == 1 ? cfg->init[live_ids[c]] : oracle_random_init(cfg->seed, trial, c, m);
        if (v == 0) x0[c >> 6] |= 1ull << (c & 63);
        else if (v == 1) x1[c >> 6] |= 1ull << (c & 63);
        if (node_out) node_out[live_ids[c]].x = (int8_t)v;
    }
    if ((int64_t)m < quorum) {          /* fewer live senders than the quorum: no trigger ever fires */
        if (node_out) {
            for (uint32_t c = 0; c < m; ++c) { node_out[live_ids[c]].k = 1; }
        }
        hist[2]++;
        return;
    }
    uint32_t R = 0;
    int all_dec = 0;
    for (uint32_t r = 1; r <= cfg->k_max; ++r) {
        /* R-phase (node.ts:52-69): every live receiver tallies all m live senders. */
        for (uint32_t w = 0; w < W; ++w) { p0[w] = p1[w] = 0; }
        for (uint32_t c = 0; c < m; ++c) {
            const uint64_t *a0 = x0, *a1 = x1;
            __asm__ volatile("" : "+r"(a0), "+r"(a1));   /* per-receiver tally: no hoisting */
            int c0 = 0, c1 = 0;
            if (cfg->mode == 1) {
                uint64_t D[64];
                oracle_delivery_mask(cfg->seed, trial, live_ids[c], r, 0, m, (uint32_t)quorum, D);
                for (uint32_t w = 0; w < W; ++w) { c0 += popc64(a0[w] & D[w]); c1 += popc64(a1[w] & D[w]); }
            } else
            for (uint32_t w = 0; w < W; ++w) { c0 += popc64(a0[w]); c1 += popc64(a1[w]); }
            if (c0 > c1) p0[c >> 6] |= 1ull << (c & 63);
            else if (c1 > c0) p1[c >> 6] |= 1ull << (c & 63);
        }
        /* P-phase (node.ts:88-113) */
        uint64_t nx0[64], nx1[64];
        for (uint32_t w = 0; w < W; ++w) { nx0[w] = nx1[w] = 0; }
        for (uint32_t c = 0; c < m; ++c) {
            const uint64_t *a0 = p0, *a1 = p1;
            __asm__ volatile("" : "+r"(a0), "+r"(a1));
            int c0 = 0, c1 = 0;
            if (cfg->mode == 1) {
                uint64_t D[64];
                oracle_delivery_mask(cfg->seed, trial, live_ids[c], r, 1, m, (uint32_t)quorum, D);
                for (uint32_t w = 0; w < W; ++w) { c0 += popc64(a0[w] & D[w]); c1 += popc64(a1[w] & D[w]); }
            } else
            for (uint32_t w = 0; w < W; ++w) { c0 += popc64(a0[w]); c1 += popc64(a1[w]); }
            int x;
            uint64_t bit = 1ull << (c & 63);
            if (c0 > (int)F) { x = 0; dec[c >> 6] |= bit; }
            else if (c1 > (int)F) { x = 1; dec[c >> 6] |= bit; }
            else if (c0 + c1 > 0 && c0 > c1) x = 0;
            else if (c0 + c1 > 0 && c0 < c1) x = 1;
            else x = oracle_coin(cfg->seed, trial, c, r);
            if (x) nx1[c >> 6] |= bit; else nx0[c >> 6] |= bit;
        }
        for (uint32_t w = 0; w < W; ++w) { x0[w] = nx0[w]; x1[w] = nx1[w]; }
        R = r;
        all_dec = 1;
        for (uint32_t w = 0; w < W; ++w) {
            uint32_t lo = w * 64, n = (m - lo) < 64 ? (m - lo) : 64;
            uint64_t vm = n == 64 ? ~0ull : ((1ull << n) - 1);
            if ((dec[w] & vm) != vm) { all_dec = 0; break; }
        }
        if (all_dec) break;
    }
    /* common value */
    int any0 = 0, any1 = 0;
    for (uint32_t w = 0; w < W; ++w) { any0 |= x0[w] != 0; any1 |= x1[w] != 0; }
    int v = (any0 && any1) ? 2 : any1 ? 1 : 0;
    if (all_dec) {
        hist[(size_t)R * 3 + (size_t)v]++;
        if (v == 2) hist[H]++;
    } else {
        hist[v]++;
    }
    if (node_out) {
        for (uint32_t c = 0; c < m; ++c) {
            orc_node_state *s = &node_out[live_ids[c]];
            uint64_t bit = 1ull << (c & 63);
            s->x = (x1[c >> 6] & bit) ? 1 : 0;
            s->decided = (dec[c >> 6] & bit) ? 1 : 0;
            s->k = (int32_t)R + 1;
        }
    }
}

/* Batch of independent trials; hist has (k_max+1)*3+1 entries (accumulated).
 * node_out (optional, only when trial_count == 1): per-node final state.
 * Returns 0, or -1 on bad config. */
int oracle_run_trials(const orc_trials_cfg *cfg, uint64_t *hist, orc_node_state *node_out) {
    if (cfg->k_max < 1 || cfg->N > 4096) return -1;
    uint32_t *live_ids = (uint32_t *)malloc(sizeof(uint32_t) * (cfg->N + 1));
    uint32_t m = 0;
    for (uint32_t i = 0; i < cfg->N; ++i) if (!cfg->faulty[i]) live_ids[m++] = i;
    /* lockstep covers the reference's admissible inputs: exactly F crash faults
     * (launchNodes.ts:12-13), or fewer live nodes than the quorum (stall).
     * f < F needs the random-delivery model (mode 1). */
    if (cfg->mode == 0 && (int64_t)m > (int64_t)cfg->N - (int64_t)cfg->F) { free(live_ids); return -2; }
    if (cfg->mode > 1) { free(live_ids); return -1; }
    if (node_out) {
        for (uint32_t i = 0; i < cfg->N; ++i) {
            int f = cfg->faulty[i] != 0;
            node_out[i].killed = (int8_t)f;
            node_out[i].x = f ? -1 : (cfg->init_mode == 1 ? cfg->init[i] : -1);
            node_out[i].decided = f ? -1 : 0;
            node_out[i].k = f ? -1 : 0;
            node_out[i].pad = 0;
        }
    }
    const size_t HS = (size_t)(cfg->k_max + 1) * 3 + 1;
    int nthreads = 1;
#ifdef _OPENMP
    nthreads = cfg->threads > 0 ? cfg->threads : omp_get_max_threads();
#endif
    if (node_out) nthreads = 1;
    uint64_t *hl = (uint64_t *)calloc((size_t)nthreads * HS, sizeof(uint64_t));
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        uint64_t x0[64], x1[64], p0[64], p1[64], dec[64];
        uint64_t *h = hl + (size_t)tid * HS;
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t t = 0; t < (int64_t)cfg->trial_count; ++t)
            run_one(cfg, live_ids, m, cfg->trial_begin + (uint64_t)t, x0, x1, p0, p1, dec, h,
                    node_out);
    }
    for (int t = 0; t < nthreads; ++t)
        for (size_t j = 0; j < HS; ++j) hist[j] += hl[(size_t)t * HS + j];
    free(hl);
    free(live_ids);
    return 0;
}

/* ===================================================================== */
/* (iii) event-level asynchronous mode, N <= 4096         */
/* ===================================================================== */
/* Message-granular restatement of node.ts:43-199 with the reference's own
 * mid-run crash: GET /stop (node.ts:191-194) may hit a live node at any
 * moment.  Per trial:
 *   - /start (node.ts:167-188): every running node sets k = 1 and broadcasts
 *     its x to all N nodes, in node order;
 *   - events e = 0, 1, ...: first every scheduled /stop with crash_at[i] == e
 *     is applied (node i killed, its x/decided/k kept), then one pending
 *     message is delivered: index = (hi32(splitmix64) * len) >> 32 over the
 *     pool, removed by swap-with-last; splitmix64 state =
 *     (philox(ctr {trial, 0, 3<<24})[0] << 32 | [1]) ^ 0xD1B54A32D192ED03;
 *   - delivery follows node.ts:45-158 literally (killed receivers drop,
 *     `>= N-F` triggers, broadcasts to all N nodes);
 *   - halting: round K is complete when every non-killed node has finished
 *     its round-K P-phase; the network stops at the first complete round in
 *     which every non-killed node has decided, or at round k_max, or when no
 *     message is left (a stall: fewer than N-F senders remain).
 * Random crash schedule (crash_at == NULL, crash_count > 0): Philox stream 4
 * (ctr {trial, block << 12, 4 << 24}, words in order) picks crash_count
 * distinct live nodes by Floyd's algorithm over compact live indices, then
 * one uniform event index in [0, crash_window) per pick, in pick order. */
typedef struct {
    uint32_t N, F, k_max, init_mode;
    uint64_t seed, trial_begin, trial_count;
    const uint8_t *faulty;
    const int8_t *init;
    const uint32_t *crash_at;       /* [N] or NULL; UINT32_MAX = never */
    uint32_t crash_count, crash_window;
    int32_t threads;
} orc_event_cfg;

#define ORC_STREAM_CRASH 4u

typedef struct { int16_t c0, c1, len, pad; } orc_ibox;

static int cmp_u64(const void *a, const void *b) {
    const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

/* bitsets over node ids (N <= ORC_EV_MAX_N) */
#define ORC_EV_MAX_N 4096u
#define ORC_EV_NW (ORC_EV_MAX_N / 64u)
typedef struct { uint64_t w[ORC_EV_NW]; } orc_set;
static inline int set_has(const orc_set *s, uint32_t i) { return (int)((s->w[i >> 6] >> (i & 63u)) & 1u); }
static inline void set_add(orc_set *s, uint32_t i) { s->w[i >> 6] |= 1ull << (i & 63u); }
static uint32_t ev_nw = ORC_EV_NW;        /* words in use: ceil(N / 64) (set per trial, below) */
#ifdef _OPENMP
#pragma omp threadprivate(ev_nw)
#endif
static inline int set_union_full(const orc_set *a, const orc_set *b, const orc_set *all) {
    for (uint32_t j = 0; j < ev_nw; ++j) if ((a->w[j] | b->w[j]) != all->w[j]) return 0;
    return 1;
}

/* One trial.  Returns the outcome bin (index into the histogram) and fills
 * state_out[N] when given; *events_out = messages delivered.  max_events <
 * UINT64_MAX truncates the run before delivery max_events (after the stops
 * scheduled there): the states of a GET /getState served at that point of a
 * live run (bo_get_states), if the run has not halted by then. */
static uint32_t event_trial(const orc_event_cfg *cfg, uint64_t trial, orc_node_state *st_out,
                            uint64_t *events_out, uint64_t max_events) {
    const uint32_t N = cfg->N, F = cfg->F, KR = cfg->k_max + 3;
    const int64_t quorum = (int64_t)N - (int64_t)F;
    orc_node_state *st = (orc_node_state *)malloc(sizeof(orc_node_state) * N);
    uint32_t *live_ids = (uint32_t *)malloc(sizeof(uint32_t) * N), *cidx = (uint32_t *)malloc(sizeof(uint32_t) * N);
    uint32_t m = 0;
    orc_set killed, decided, all;
    ev_nw = (N + 63u) / 64u;
    memset(&killed, 0, sizeof killed);
    memset(&decided, 0, sizeof decided);
    memset(&all, 0, sizeof all);
    for (uint32_t i = 0; i < N; ++i) {
        const int f = cfg->faulty[i] != 0;
        st[i].killed = (int8_t)f; st[i].decided = f ? -1 : 0; st[i].k = f ? -1 : 0; st[i].pad = 0;
        st[i].x = -1;
        cidx[i] = m;
        set_add(&all, i);
        if (f) set_add(&killed, i); else live_ids[m++] = i;
    }
    for (uint32_t c = 0; c < m; ++c) {
        const uint32_t i = live_ids[c];
        st[i].x = (int8_t)(cfg->init_mode == 1 ? cfg->init[i] : oracle_random_init(cfg->seed, trial, c, m));
    }
    /* crash schedule */
    uint32_t *crash_at = (uint32_t *)malloc(sizeof(uint32_t) * N);
    for (uint32_t i = 0; i < N; ++i) crash_at[i] = cfg->crash_at ? cfg->crash_at[i] : 0xFFFFFFFFu;
    if (!cfg->crash_at && cfg->crash_count > 0 && m > 0 && cfg->crash_window > 0) {
        orc_dstream s;
        s.key[0] = (uint32_t)cfg->seed; s.key[1] = (uint32_t)(cfg->seed >> 32);
        s.ctr[0] = (uint32_t)trial; s.ctr[1] = (uint32_t)(trial >> 32);
        s.ctr[2] = 0; s.ctr[3] = ORC_STREAM_CRASH << 24; s.widx = 0; s.blk_shift = 12;
        const uint32_t k = cfg->crash_count < m ? cfg->crash_count : m;
        orc_set T;
        memset(&T, 0, sizeof T);
        uint32_t *picks = (uint32_t *)malloc(sizeof(uint32_t) * (k + 1));
        for (uint32_t j = m - k, n = 0; j < m; ++j, ++n) {
            const uint32_t t = dstream_uniform(&s, j + 1u);
            const uint32_t idx = set_has(&T, t) ? j : t;
            set_add(&T, idx);
            picks[n] = idx;
        }
        for (uint32_t n = 0; n < k; ++n) crash_at[live_ids[picks[n]]] = dstream_uniform(&s, cfg->crash_window);
        free(picks);
    }
    /* inboxes[node][k][phase] */
    orc_ibox *ib = (orc_ibox *)calloc((size_t)N * KR * 2, sizeof(orc_ibox));
    orc_set *comp = (orc_set *)calloc(KR, sizeof(orc_set));
    uint8_t *pdone = (uint8_t *)calloc((size_t)N * KR, 1);
    size_t cap = (size_t)4 * N * N + 64, len = 0;
    uint32_t *pool = (uint32_t *)malloc(cap * sizeof(uint32_t));
    /* message: to (12 bits) | phase << 12 | (x & 3) << 13 | k << 15 */
#define EV_SEND(K, X, PH)                                                               \
    do {                                                                                \
        for (uint32_t to_ = 0; to_ < N; ++to_) {                                        \
            if (len == cap) { cap *= 2; pool = (uint32_t *)realloc(pool, cap * 4); }   \
            pool[len++] = to_ | ((uint32_t)(PH) << 12) | ((uint32_t)((X) & 3) << 13) | ((uint32_t)(K) << 15); \
        }                                                                               \
    } while (0)
    orc_rng rng;
    rng.s = (((uint64_t)orc_philox_word(cfg->seed, trial, 0, ORC_STREAM_ORDER << 24, 0) << 32) |
             orc_philox_word(cfg->seed, trial, 0, ORC_STREAM_ORDER << 24, 1)) ^ 0xD1B54A32D192ED03ull;
    for (uint32_t i = 0; i < N; ++i)                    /* /start, node.ts:171-185 */
        if (!set_has(&killed, i)) { st[i].k = 1; EV_SEND(1u, st[i].x, 0u); }
    uint32_t cur = 1, R = 0;
    int halted = 0;                                      /* 1 decided, 2 k_max, 3 stall */
    uint64_t e = 0;
    /* the schedule as (event, node) pairs in ascending order: the stops of
     * event e are applied in node order, as a scan over i would */
    uint64_t *stops = (uint64_t *)malloc(sizeof(uint64_t) * (N + 1));
    uint32_t n_stops = 0, next_stop = 0;
    for (uint32_t i = 0; i < N; ++i)
        if (crash_at[i] != 0xFFFFFFFFu) stops[n_stops++] = ((uint64_t)crash_at[i] << 32) | i;
    qsort(stops, n_stops, sizeof(uint64_t), cmp_u64);
    for (;;) {
        /* scheduled /stop (node.ts:191-194) */
        int crashed = 0;
        for (; next_stop < n_stops && (stops[next_stop] >> 32) == e; ++next_stop) {
            const uint32_t i = (uint32_t)stops[next_stop];
            if (!set_has(&killed, i)) { set_add(&killed, i); st[i].killed = 1; crashed = 1; }
        }
        if (crashed && set_union_full(&killed, &killed, &all)) { halted = 3; break; }
        if (crashed) {
            while (cur < KR && set_union_full(&comp[cur], &killed, &all)) {
                if (set_union_full(&decided, &killed, &all)) { halted = 1; R = cur; break; }
                if (cur >= cfg->k_max) { halted = 2; R = cur; break; }
                ++cur;
            }
            if (halted) break;
        }
        if (e >= max_events) break;                      /* a snapshot of the running network */
        if (len == 0) { halted = 3; break; }
        const uint32_t pick = (uint32_t)(((uint64_t)(uint32_t)(orc_splitmix(&rng) >> 32) * (uint64_t)len) >> 32);
        const uint32_t msg = pool[pick];
        pool[pick] = pool[--len];
        ++e;
        const uint32_t to = msg & 4095u, ph = (msg >> 12) & 1u, k = msg >> 15;
        const int8_t x = (int8_t)((msg >> 13) & 3u);
        if (set_has(&killed, to)) continue;              /* node.ts:45 */
        if (k >= KR) continue;
        orc_ibox *b = &ib[((size_t)to * KR + k) * 2 + ph];
        b->len++;
        if (x == 0) b->c0++; else if (x == 1) b->c1++;
        if ((int64_t)b->len < quorum) continue;          /* node.ts:52, :88 */
        const int c0 = b->c0, c1 = b->c1;
        if (ph == 0) {                                   /* node.ts:53-80 */
            const int8_t v = (c0 > c1) ? 0 : (c1 > c0) ? 1 : 2;
            EV_SEND(k, v, 1u);
        } else {                                         /* node.ts:89-157 */
            if (c0 > (int)F) { st[to].x = 0; st[to].decided = 1; set_add(&decided, to); }
            else if (c1 > (int)F) { st[to].x = 1; st[to].decided = 1; set_add(&decided, to); }
            else if (c0 + c1 > 0 && c0 > c1) st[to].x = 0;
            else if (c0 + c1 > 0 && c0 < c1) st[to].x = 1;
            else st[to].x = (int8_t)oracle_coin(cfg->seed, trial, cidx[to], k);
            st[to].k = (int32_t)k + 1;
            uint8_t *pd = &pdone[(size_t)to * KR + k];
            if (!*pd) {
                *pd = 1;
                set_add(&comp[k], to);
                while (cur < KR && set_union_full(&comp[cur], &killed, &all)) {
                    if (set_union_full(&decided, &killed, &all)) { halted = 1; R = cur; break; }
                    if (cur >= cfg->k_max) { halted = 2; R = cur; break; }
                    ++cur;
                }
                if (halted) break;
            }
            EV_SEND(k + 1, st[to].x, 0u);
        }
    }
#undef EV_SEND
    free(ib); free(comp); free(pdone); free(pool); free(crash_at); free(stops);
    if (events_out) *events_out = e;
    /* outcome over the nodes still running */
    int any0 = 0, any1 = 0, anyq = 0, nlive = 0;
    for (uint32_t i = 0; i < N; ++i) {
        if (set_has(&killed, i)) continue;
        ++nlive;
        if (st[i].x == 0) any0 = 1; else if (st[i].x == 1) any1 = 1; else anyq = 1;
    }
    const uint32_t v = (nlive == 0 || anyq || (any0 && any1)) ? 2u : (any1 ? 1u : 0u);
    if (st_out) for (uint32_t i = 0; i < N; ++i) st_out[i] = st[i];
    free(st); free(live_ids); free(cidx);
    if (halted == 1) return (uint32_t)((size_t)R * 3 + v) | (v == 2 ? 0x80000000u : 0u);
    return v;
}

/* Batch: hist as oracle_run_trials; events_out (optional) = total messages delivered. */
int oracle_event_trials(const orc_event_cfg *cfg, uint64_t *hist, orc_node_state *node_out, uint64_t *events_out) {
    if (cfg->k_max < 1 || cfg->N < 1 || cfg->N > ORC_EV_MAX_N) return -1;
    uint32_t f = 0;
    for (uint32_t i = 0; i < cfg->N; ++i) f += cfg->faulty[i] ? 1 : 0;
    if (f != cfg->F) return -2;                          /* launchNodes.ts:12-13 */
    const size_t HS = (size_t)(cfg->k_max + 1) * 3 + 1;
    uint64_t ev = 0;
    int nthreads = 1;
#ifdef _OPENMP
    nthreads = cfg->threads > 0 ? cfg->threads : omp_get_max_threads();
#endif
    if (node_out) nthreads = 1;
    uint64_t *hl = (uint64_t *)calloc((size_t)nthreads * HS, sizeof(uint64_t));
    uint64_t *el = (uint64_t *)calloc((size_t)nthreads, sizeof(uint64_t));
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads) schedule(static)
#endif
    for (int64_t t = 0; t < (int64_t)cfg->trial_count; ++t) {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        uint64_t e = 0;
        const uint32_t bin = event_trial(cfg, cfg->trial_begin + (uint64_t)t, node_out, &e, UINT64_MAX);
        hl[(size_t)tid * HS + (bin & 0x7FFFFFFFu)]++;
        if (bin & 0x80000000u) hl[(size_t)tid * HS + HS - 1]++;
        el[tid] += e;
    }
    for (int t = 0; t < nthreads; ++t) {
        for (size_t j = 0; j < HS; ++j) hist[j] += hl[(size_t)t * HS + j];
        ev += el[t];
    }
    free(hl); free(el);
    if (events_out) *events_out = ev;
    return 0;
}

/* The per-node states of trial `trial` before delivery max_events (a live
 * run's GET /getState snapshot, include/benor.h bo_get_states); *halted_out =
 * 1 when the run halted before reaching that count (the states are then the
 * final ones).  *events_out = deliveries made. */
int oracle_event_states_at(const orc_event_cfg *cfg, uint64_t trial, uint64_t max_events, orc_node_state *st_out,
                           uint64_t *events_out) {
    if (cfg->k_max < 1 || cfg->N < 1 || cfg->N > ORC_EV_MAX_N || !st_out) return -1;
    uint32_t f = 0;
    for (uint32_t i = 0; i < cfg->N; ++i) f += cfg->faulty[i] ? 1 : 0;
    if (f != cfg->F) return -2;                          /* launchNodes.ts:12-13 */
    uint64_t e = 0;
    (void)event_trial(cfg, trial, st_out, &e, max_events);
    if (events_out) *events_out = e;
    return 0;
}
