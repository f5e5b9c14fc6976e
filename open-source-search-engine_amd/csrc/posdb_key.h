// Posdb key codec shared by the host library and the HIP kernels.
//
// An 18-byte posdb key (Posdb.h:3-25, key144_t types.h:431-475) is stored
// little-endian as n0 (u16, bytes 0-1), n1 (u64, bytes 2-9), n2 (u64, 10-17):
//
//   n2: termId(48) | docId[37:22](16)
//   n1: docId[21:0](22) | 0 | siteRank(4) | langId[4:0](5) | wordPos(18) |
//       hashGroup(4) | wordSpamRank(4) | diversityRank(4) | F(2)
//   n0: densityRank(5) | b | 1 | multiplier(5) | langId[5] | comp(2) | del
//
// Lists are compressed on append (RdbList.cpp:282-327): a key whose top 6
// bytes (termId) and middle 6 bytes (docId/siteRank/langId) repeat the
// previous key is stored as its low 6 bytes with byte0 |= 0x06; a key whose
// termId repeats is stored as its low 12 bytes with byte0 |= 0x02.
//
// Every key start has byte1 & 0x02 set (the n0 "1" bit); the second half of
// a 12-byte key has byte 7 & 0x02 clear (the n1 zero bit, Posdb.cpp:410-412).
// That lets each 6-byte unit of a list be classified without a serial walk.
#ifndef GBGPU_POSDB_KEY_H
#define GBGPU_POSDB_KEY_H

#include <stdint.h>

#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define GB_HD __host__ __device__ __forceinline__
#else
#define GB_HD static inline
#endif

#define GB_MAXSITERANK      0x0f
#define GB_MAXLANGID        0x3f
#define GB_MAXWORDPOS       0x0003ffff
#define GB_MAXDENSITYRANK   0x1f
#define GB_MAXWORDSPAMRANK  0x0f
#define GB_MAXDIVERSITYRANK 0x0f
#define GB_MAXHASHGROUP     0x0f
#define GB_MAXMULTIPLIER    0x0f

// hash groups (Posdb.h:73-84)
#define GB_HG_BODY               0
#define GB_HG_TITLE              1
#define GB_HG_HEADING            2
#define GB_HG_INLIST             3
#define GB_HG_INMETATAG          4
#define GB_HG_INLINKTEXT         5
#define GB_HG_INTAG              6
#define GB_HG_NEIGHBORHOOD       7
#define GB_HG_INTERNALINLINKTEXT 8
#define GB_HG_INURL              9
#define GB_HG_INMENU             10
#define GB_HG_END                11

GB_HD uint32_t gb_u16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
GB_HD uint32_t gb_u32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// getKeySize (Posdb.h:271-275)
GB_HD int gb_key_size(const uint8_t *k) { return (k[0] & 0x04) ? 6 : ((k[0] & 0x02) ? 12 : 18); }
// getDocId (Posdb.h:295-306): LE40(bytes 7..11) >> 2
GB_HD uint64_t gb_docid(const uint8_t *k) {
  uint64_t d = (uint64_t)k[11];
  d = (d << 32) | gb_u32(k + 7);
  return d >> 2;
}
// "docid key" used by the vote buffer compare (Posdb.cpp:5100-5113): u32 at
// +8 then byte7 & 0xfc.  Equal ordering to gb_docid.
GB_HD uint32_t gb_wordpos(const uint8_t *k) { return gb_u32(k + 2) >> 14; }       // Posdb.h:324
GB_HD uint32_t gb_hashgroup(const uint8_t *k) { return (k[3] >> 2) & 0x0f; }       // Posdb.h:319
GB_HD uint32_t gb_wordspam(const uint8_t *k) { return (gb_u16(k + 2) >> 6) & 0x0f; } // Posdb.h:341
GB_HD uint32_t gb_diversity(const uint8_t *k) { return (k[2] >> 2) & 0x0f; }       // Posdb.h:346
GB_HD uint32_t gb_is_syn(const uint8_t *k) { return k[2] & 0x03; }                  // Posdb.h:351
GB_HD uint32_t gb_is_hswb(const uint8_t *k) { return k[2] & 0x01; }                 // Posdb.h:355
GB_HD uint32_t gb_density(const uint8_t *k) { return (gb_u16(k) >> 11) & 0x1f; }    // Posdb.h:359
GB_HD uint32_t gb_multiplier(const uint8_t *k) { return (gb_u16(k) >> 4) & 0x0f; }  // Posdb.h:379
GB_HD uint32_t gb_siterank(const uint8_t *k) {                                      // Posdb.h:308
  return ((uint32_t)(k[6] >> 5) | ((uint32_t)(k[7] & 1) << 3)) & 0x0f;
}
GB_HD uint32_t gb_langid(const uint8_t *k) {                                        // Posdb.h:312
  return (uint32_t)(k[6] & 0x1f) | ((k[0] & 0x08) ? 0x20u : 0u);
}
GB_HD uint64_t gb_termid(const uint8_t *k) {                                        // Posdb.h:291
  uint64_t t = 0;
  for (int i = 5; i >= 0; i--) t = (t << 8) | k[12 + i];
  return t;
}
// 6-byte unit classification: key start?  (Posdb.h:887-889 b-step idiom)
GB_HD int gb_unit_is_key_start(const uint8_t *u) { return (u[1] & 0x02) != 0; }
// key start that opens a docid run (12- or 18-byte key)
GB_HD int gb_unit_is_run_start(const uint8_t *u) { return (u[1] & 0x02) && !(u[0] & 0x04); }

#define GB_TERMID_MASK 0x0000ffffffffffffULL
#define GB_DOCID_MASK  0x0000003fffffffffULL

// Posdb::makeKey (Posdb.cpp:374-460) into 18 little-endian bytes.
GB_HD void gb_make_key(uint8_t *out, uint64_t termId, uint64_t docId, uint32_t wordPos,
                       uint32_t densityRank, uint32_t diversityRank, uint32_t wordSpamRank,
                       uint32_t siteRank, uint32_t hashGroup, uint32_t langId,
                       uint32_t multiplier, int isSynonym, int isDelKey, int shardByTermId) {
  uint64_t n2 = (termId & GB_TERMID_MASK);
  n2 <<= 16;
  n2 |= docId >> 22;
  uint64_t n1 = docId & 0x3fffff;
  n1 <<= 1;
  n1 <<= 4; n1 |= siteRank;
  n1 <<= 5; n1 |= (langId & 0x1f);
  n1 <<= 18; n1 |= wordPos;
  n1 <<= 4; n1 |= hashGroup;
  n1 <<= 4; n1 |= wordSpamRank;
  n1 <<= 4; n1 |= diversityRank;
  n1 <<= 2; if (isSynonym) n1 |= 0x01;
  uint32_t n0 = densityRank;
  n0 <<= 1;
  n0 <<= 1; n0 |= 0x01;
  n0 <<= 5; n0 |= multiplier;
  n0 <<= 1; if (langId & 0x20) n0 |= 0x01;
  n0 <<= 2;
  n0 <<= 1; if (!isDelKey) n0 |= 0x01;
  n0 &= 0xffff;
  out[0] = (uint8_t)n0; out[1] = (uint8_t)(n0 >> 8);
  for (int i = 0; i < 8; i++) out[2 + i] = (uint8_t)(n1 >> (8 * i));
  for (int i = 0; i < 8; i++) out[10 + i] = (uint8_t)(n2 >> (8 * i));
  if (shardByTermId) out[1] |= 0x01;
}

#endif
