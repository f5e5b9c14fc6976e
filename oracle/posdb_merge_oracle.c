/* TEST INFRASTRUCTURE ONLY (see posdb_oracle.h).
 *
 * Restatement of RdbList::posdbMerge_r (RdbList.cpp:3065-3568) with the
 * bfcmpPosdb comparator (RdbList.h:620-641), for lists already prepared by
 * prepareForMerge (every input list starts with an 18-byte key) merging into
 * an empty output list.  Pinned bit-exact against the reference's own
 * RdbList::merge_r (oracle/ref.mk, tests/golden/m_*.npz).
 */
#include "posdb_oracle.h"

#include <errno.h>
#include <string.h>

static inline uint32_t U32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint16_t U16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }

/* bfcmpPosdb, RdbList.h:620-641 */
static int bfcmpPosdb(const uint8_t *alo, const uint8_t *ame, const uint8_t *ahi, const uint8_t *blo,
                      const uint8_t *bme, const uint8_t *bhi) {
  if (U32(ahi + 2) < U32(bhi + 2)) return -1;
  if (U32(ahi + 2) > U32(bhi + 2)) return 1;
  if (U16(ahi) < U16(bhi)) return -1;
  if (U16(ahi) > U16(bhi)) return 1;
  if (U32(ame + 2) < U32(bme + 2)) return -1;
  if (U32(ame + 2) > U32(bme + 2)) return 1;
  if (U16(ame) < U16(bme)) return -1;
  if (U16(ame) > U16(bme)) return 1;
  if (U32(alo + 2) < U32(blo + 2)) return -1;
  if (U32(alo + 2) > U32(blo + 2)) return 1;
  if ((U16(alo) | 0x0007) < (U16(blo) | 0x0007)) return -1;
  if ((U16(alo) | 0x0007) > (U16(blo) | 0x0007)) return 1;
  return 0;
}

#define MAXL 256

int64_t orc_posdb_merge(const uint8_t *const *lists, const int64_t *sizes, int numLists,
                        int removeNegKeys, int64_t minRecSizes, uint8_t *out, int64_t cap) {
  if (numLists < 0 || numLists > MAXL) return -EINVAL;
  if (minRecSizes == 0) return 0;
  const int numListsIn = numLists;
  const uint8_t *ptrs[MAXL], *ends[MAXL], *hiKeys[MAXL], *loKeys[MAXL];
  int n = 0;
  for (int i = 0; i < numLists; i++) {
    if (sizes[i] <= 0) continue;
    if (lists[i][0] & 0x06) return -EINVAL; /* first key must be 18 bytes */
    ends[n] = lists[i] + sizes[i];
    ptrs[n] = lists[i];
    hiKeys[n] = lists[i] + 12;
    loKeys[n] = lists[i] + 6;
    n++;
  }
  numLists = n;
  if (numLists <= 0) return 0;
  /* prepareForMerge (RdbList.cpp:410-491) and merge_r (RdbList.cpp:1658-1756)
   * turn the caller's minRecSizes into the bound posdbMerge_r receives:
   * m_mergeMinListSize = min(sum of list sizes, minRecSizes + 2 * 18) for
   * posdb (18-byte keys, fixedDataSize 0), or the sum when minRecSizes < 0.
   * maxPtr = m_list + that, capped to the allocation (RdbList.cpp:3127-3133). */
  int64_t total = 0;
  for (int i = 0; i < numListsIn; i++) total += sizes[i] > 0 ? sizes[i] : 0;
  int64_t maxOff = total;
  if (minRecSizes > 0) {
    int64_t nm = (int64_t)(int32_t)((uint32_t)minRecSizes + 36u);
    if (nm < minRecSizes) nm = 0x7fffffff;
    if (maxOff > nm) maxOff = nm;
  }
  if (maxOff > cap) maxOff = cap;
  uint8_t *listPtr = out;
  uint8_t *listPtrLo = NULL, *listPtrHi = NULL, *pp = NULL;
  const uint8_t *minPtrBase, *minPtrLo, *minPtrHi;
  int mini;
  for (;;) {
    /* top: */
    minPtrBase = ptrs[0];
    minPtrLo = loKeys[0];
    minPtrHi = hiKeys[0];
    mini = 0;
    int tie = 0;
    for (int i = 1; i < numLists; i++) {
      int ss = bfcmpPosdb(minPtrBase, minPtrLo, minPtrHi, ptrs[i], loKeys[i], hiKeys[i]);
      if (ss < 0) continue;
      if (ss == 0) { tie = 1; break; } /* goto skip: drop the older key */
      minPtrBase = ptrs[i];
      minPtrLo = loKeys[i];
      minPtrHi = hiKeys[i];
      mini = i;
    }
    if (!tie && !(removeNegKeys && (minPtrBase[0] & 0x01) == 0x00)) {
      if (listPtr + 18 > out + cap) return -ENOSPC;
      pp = listPtr;
      memcpy(listPtr, minPtrBase, 6);
      listPtr += 6;
      int hiDiff = (!listPtrHi || U32(minPtrHi) != U32(listPtrHi) || U16(minPtrHi + 4) != U16(listPtrHi + 4));
      *pp &= 0xf9;
      if (hiDiff || !listPtrLo || U32(minPtrLo) != U32(listPtrLo) || U16(minPtrLo + 4) != U16(listPtrLo + 4)) {
        memcpy(listPtr, minPtrLo, 6);
        listPtrLo = listPtr;
        listPtr += 6;
      } else {
        *pp |= 0x06;
      }
      if (hiDiff) {
        memcpy(listPtr, minPtrHi, 6);
        listPtrHi = listPtr;
        listPtr += 6;
      } else {
        if (!(*pp & 0x04)) *pp |= 0x02;
      }
    }
    /* skip: */
    if (ptrs[mini][0] & 0x04) ptrs[mini] += 6;
    else if (ptrs[mini][0] & 0x02) ptrs[mini] += 12;
    else ptrs[mini] += 18;
    if (ptrs[mini] < ends[mini]) {
      if (ptrs[mini][0] & 0x04) {
      } else if (ptrs[mini][0] & 0x02) {
        loKeys[mini] = ptrs[mini] + 6;
      } else {
        hiKeys[mini] = ptrs[mini] + 12;
        loKeys[mini] = ptrs[mini] + 6;
      }
      if (listPtr - out >= maxOff) break;
      continue;
    }
    for (int i = mini; i < numLists - 1; i++) {
      ptrs[i] = ptrs[i + 1];
      ends[i] = ends[i + 1];
      hiKeys[i] = hiKeys[i + 1];
      loKeys[i] = loKeys[i + 1];
    }
    numLists--;
    if (listPtr - out >= maxOff) break;
    if (numLists > 0) continue;
    break;
  }
  return listPtr - out;
}
