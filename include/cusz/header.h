/* include/cusz/header.h -- the 176-byte archive header (psz_header).
 *
 * Byte layout equals the reference psz/include/cusz/header.h:19-48 (measured offsets in
 * SURVEY.md Appendix D): dtype@0 pipeline@4 rc@24 vle_sublen@48 vle_pardeg@52 entry[6]@56
 * len@80 splen@104 user_input_eb@112 min_val@120 max_val@128 intp_param@136, size 176.
 *
 * Archive = [psz_header 176 B][anchor][Huffman (phf) segment][outlier cells 8 B each];
 * entry[k] is the byte offset of segment k, entry[5] the archive size.  Unlike the
 * reference, this implementation also writes the header into the device archive and
 * defines entry[5] = entry[4] (reference reads an uninitialised nbyte[4], Appendix B.4).
 */
#ifndef CUSZ_AMD_HEADER_H
#define CUSZ_AMD_HEADER_H

#ifdef __cplusplus
extern "C" {
#endif

#include "cusz/type.h"

#define PSZHEADER_HEADER 0
#define PSZHEADER_ANCHOR 1
#define PSZHEADER_ENCODED 2
#define PSZHEADER_SPFMT 3
#define PSZHEADER_ENC_PASS1_END 4
#define PSZHEADER_ENC_PASS2_END 5

typedef struct psz_header {
  union {
    struct {
      psz_dtype dtype;
      psz_pipeline pipeline;
      psz_rc2 rc;

      int vle_sublen; /* Huffman chunk length (symbols) */
      int vle_pardeg; /* number of chunks */

      uint32_t entry[PSZHEADER_ENC_PASS2_END + 1];

      psz_len len;
      size_t splen; /* number of outlier cells */

      double user_input_eb;
      double min_val, max_val;

      INTERPOLATION_PARAMS intp_param;
    };
  };
} psz_header;

psz_len pszheader_len(psz_header*);
size_t pszheader_len_linear(psz_header*);
size_t pszheader_segments(psz_header*);
size_t pszheader_filesize(psz_header*);
size_t pszheader_uncompressed_len(psz_header*);
size_t pszheader_compressed_bytes(psz_header*);

#ifdef __cplusplus
}
#endif

#endif /* CUSZ_AMD_HEADER_H */
