/* TEST INFRASTRUCTURE ONLY: RdbList::posdbMerge_r restatement (next
 * milestone).  Parity unpinned. */
#include "posdb_oracle.h"

#include <errno.h>

int64_t orc_posdb_merge(const uint8_t *const *lists, const int64_t *sizes, int n,
                        int remove_neg_keys, int64_t min_rec_sizes, uint8_t *out, int64_t cap) {
  (void)lists; (void)sizes; (void)n; (void)remove_neg_keys; (void)min_rec_sizes; (void)out; (void)cap;
  return -ENOSYS;
}
