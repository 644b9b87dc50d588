"""Reference-format archives assembled by the CPU oracle (test infrastructure): the bytes a
reference encoder writes for given codes, outliers and codebook, at any chunk length."""
import numpy as np


def oracle_archive(oracle, codes, ol_val, ol_idx, dims, eb, book, rv, sublen, bklen=1024):
    """Reference-layout archive (psz_header | phf segment | outlier cells) from oracle codes and
    a given codebook (hf_buf.cc:191-211, compressor.inl:398-418).  dims are (x, y, z)."""
    import cusz_amd as cz

    nbit, entry, bs, tot = oracle.hf_encode(codes, book, sublen)
    pardeg = nbit.size
    sizes = [oracle.PHF_FORCED_ALIGN, rv.size, 4 * pardeg, 4 * pardeg, 4 * bs.size]
    ent = [0]
    for s in sizes:
        ent.append(ent[-1] + s)
    phf = oracle.phf_header_bytes(bklen, sublen, pardeg, codes.size, tot, bs.size, ent)
    phf += b"\0" * (oracle.PHF_FORCED_ALIGN - len(phf)) + rv.tobytes() + nbit.tobytes() + \
        entry.tobytes() + bs.tobytes()
    cells = np.empty((ol_idx.size, 2), np.uint32)
    cells[:, 0] = np.asarray(ol_val, np.float32).view(np.uint32)
    cells[:, 1] = ol_idx
    h = cz.psz_header()
    h.dtype, h.pipeline.predictor, h.pipeline.codec1 = cz.F4, cz.Lorenzo, cz.Huffman
    h.rc.mode, h.rc.eb, h.rc.radius = cz.Abs, eb, bklen // 2
    h.vle_sublen, h.vle_pardeg = sublen, pardeg
    h.len.x, h.len.y, h.len.z = dims
    h.splen = ol_idx.size
    h.user_input_eb = eb
    e = [0, 176, 176, 176 + len(phf), 176 + len(phf) + 8 * ol_idx.size, 176 + len(phf) + 8 * ol_idx.size]
    for i, v in enumerate(e):
        h.entry[i] = v
    return bytes(h) + phf + cells.tobytes()
