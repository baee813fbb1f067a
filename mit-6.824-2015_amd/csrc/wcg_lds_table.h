// wcg_lds_table.h - exact-key hash table in LDS (one per workgroup), 2-choice x 4-way buckets.
//
// Keys are the fixed-width inline identities of fact F4 (k0 = bytes 0-7, k1 = bytes 8-14 |
// len << 56, never 0).  A key may occupy one of 8 slots: 4 in bucket b1 (hash bits 32-63) and
// 4 in bucket b2 (bits 0-31).  Lookup reads the 4 first-words of a bucket with two
// ds_read_b128; insertion claims an empty slot with a 64-bit LDS CAS on k0 and then publishes
// k1.  Two lanes inserting the same new key at the same moment can end up in two different
// slots: that duplicate is harmless (both counts are flushed and summed downstream), so no lane
// ever waits for another lane's publish.
#pragma once
#include "wcg_common.h"

namespace wcg {

template <int NB, typename CNT>
struct LdsTable {
    u64 (*k0)[4];
    u64 (*k1)[4];
    CNT (*cnt)[4];

    __device__ __forceinline__ void init(int tid, int nt) {
        for (int i = tid; i < NB * 4; i += nt) {
            (&k0[0][0])[i] = 0;
            (&k1[0][0])[i] = 0;
            (&cnt[0][0])[i] = 0;
        }
    }

    __device__ __forceinline__ static void buckets(u32 h, u32& b1, u32& b2) {
        b1 = __umulhi(h, (u32)NB);
        b2 = __umulhi(__builtin_rotateleft32(h, 16), (u32)NB);
        if (b2 == b1) b2 = (b1 + 1 == (u32)NB) ? 0 : b1 + 1;
    }

    __device__ __forceinline__ void add_cnt(u32 b, int j, CNT c) { atomicAdd(&cnt[b][j], c); }

    __device__ __forceinline__ void read4(u32 b, u64 (&v)[4]) const {
        const uint4* p = reinterpret_cast<const uint4*>(&k0[b][0]);
        uint4 x = p[0], y = p[1];
        v[0] = (u64)x.y << 32 | x.x; v[1] = (u64)x.w << 32 | x.z;
        v[2] = (u64)y.y << 32 | y.x; v[3] = (u64)y.w << 32 | y.z;
    }

    // aggregate (key, c) with h = lds_hash(key); false when both buckets hold other keys.
    // Straight-line common path: both buckets are read, the 8 candidate slots become bit
    // masks (slot s: bucket s >> 2, way s & 3), one LDS atomic at a computed address.
    __device__ __forceinline__ bool add(u64 a0, u64 a1, u32 h, CNT c) {
        u32 b1, b2;
        buckets(h, b1, b2);
        const bool shrt = key_short(a0);
        u64 v[4], w[4];
        read4(b1, v);
        read4(b2, w);
        u32 m = 0, e = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            m |= (u32)(v[j] == a0) << j;
            m |= (u32)(w[j] == a0) << (4 + j);
            e |= (u32)(v[j] == 0) << j;
            e |= (u32)(w[j] == 0) << (4 + j);
        }
        if (!shrt && m) {                       // keys of 8+ bytes: confirm k1 (usually 1 candidate)
            u32 mm = m;
            m = 0;
            while (mm) {
                const int s = __ffs(mm) - 1;
                mm &= mm - 1;
                if (k1[s < 4 ? b1 : b2][s & 3] == a1) { m = 1u << s; break; }
            }
        }
        if (m) {
            const int s = __ffs(m) - 1;
            add_cnt(s < 4 ? b1 : b2, s & 3, c);
            return true;
        }
        while (e) {                             // insert: first empty slot of b1, then b2
            const int s = __ffs(e) - 1;
            e &= e - 1;
            const u32 b = s < 4 ? b1 : b2;
            const int j = s & 3;
            const u64 old = atomicCAS(&k0[b][j], 0ull, a0);
            if (old == 0) {
                if (!shrt) k1[b][j] = a1;
                add_cnt(b, j, c);
                return true;
            }
            if (old == a0 && (shrt || k1[b][j] == a1)) { add_cnt(b, j, c); return true; }
        }
        return false;
    }
};

// Hash-derived indices shared by every kernel that touches a key (they must agree):
//   LDS buckets: lds_hash (LdsTable::buckets)
//   miss-log bucket and global slot: key_hash, an independent function, so a miss bucket's
//   keys spread over the whole LDS table of the aggregation kernel.
//   h2 = key_hash(k0, k1): miss bucket = low bits, global slot = bits 16+
__device__ __forceinline__ u32 miss_bucket(u64 h2, u32 pmask) { return (u32)h2 & pmask; }
__device__ __forceinline__ u64 gslot(u64 h2) { return h2 >> 16; }

// Miss-log entries are 16 bytes {k0, k1}.  A flushed LDS slot with count > 1 is written as
// {k0, k1 | CNT_FLAG} followed by the carrier {0, count} (k0 == 0 marks a carrier / filler).
constexpr u64 CNT_FLAG = 1ull << 63;

}  // namespace wcg
