// revcomp_kernel.hip -- reverseComplement.c:21-118 as data-parallel byte
// kernels (HBM-bound map + scans).  Included by imsame_dev.hip.
//
// Semantics restated:
//  * every '>' byte opens a record (:48-54); records are emitted last first (:56)
//  * header = bytes from the '>' through the first '\n' (fgets, :59-62)
//  * body   = bytes after the header up to the next '>' (:64-70); only
//    letters (isupper || islower) are kept, reversed, complemented
//    A<->T C<->G U->A, case kept, other letters unchanged (:71-106)
//  * one '\n' after each record's sequence (:109-110)
// Records whose '>' sits inside another header share that header's body.

__device__ __forceinline__ bool rc_is_letter(uint8_t c) { return (uint8_t)((c | 0x20) - 'a') < 26u; }

__device__ __forceinline__ uint8_t rc_comp(uint8_t c) {
    switch (c) {
    case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A'; case 'U': return 'A';
    case 'a': return 't'; case 'c': return 'g'; case 'g': return 'c'; case 't': return 'a'; case 'u': return 'a';
    }
    return c;
}

// per byte: '>' flag and letter flag (inputs of two scans)
__global__ void rc_flags(const uint8_t *in, uint64_t n, uint32_t *fgt, uint32_t *flet) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t c = in[i];
    fgt[i] = c == '>';
    flet[i] = rc_is_letter(c);
}

__global__ void rc_offsets(const uint8_t *in, uint64_t n, const uint32_t *gpos, uint32_t *off) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n && in[i] == '>') off[gpos[i]] = (uint32_t)i;
}

// per record k: header end (exclusive, after '\n'), body end, sizes
__global__ void rc_records(const uint8_t *in, uint64_t n, const uint32_t *off, uint32_t nr, const uint32_t *let,
                           uint32_t *hend, uint32_t *bend, uint32_t *size_rev) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nr) return;
    uint64_t h = off[k];
    while (h < n && in[h] != '\n') ++h;
    if (h < n) ++h;
    uint32_t lo = 0, hi = nr;                  // first record offset >= h
    while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (off[m] < h) lo = m + 1; else hi = m; }
    const uint64_t b = lo < nr ? off[lo] : n;
    hend[k] = (uint32_t)h;
    bend[k] = (uint32_t)b;
    const uint32_t letters = let[b] - let[h];
    size_rev[nr - 1 - k] = (uint32_t)(h - off[k]) + letters + 1;
}

__global__ void rc_headers(const uint8_t *in, const uint32_t *off, uint32_t nr, const uint32_t *hend,
                           const uint32_t *bend, const uint32_t *let, const uint32_t *oo, uint8_t *out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nr) return;
    const uint32_t o = oo[nr - 1 - k];
    uint32_t w = 0;
    for (uint32_t h = off[k]; h < hend[k]; ++h) out[o + w++] = in[h];
    out[o + w + (let[bend[k]] - let[hend[k]])] = '\n';
}

// every body letter goes to each record whose body contains it
__global__ void rc_bodies(const uint8_t *in, uint64_t n, const uint32_t *off, uint32_t nr, const uint32_t *hend,
                          const uint32_t *bend, const uint32_t *let, const uint32_t *oo, uint8_t *out) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n || nr == 0) return;
    const uint8_t c = in[i];
    if (!rc_is_letter(c)) return;
    uint32_t lo = 0, hi = nr;                  // last record with hend <= i
    while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (hend[m] <= i) lo = m + 1; else hi = m; }
    if (lo == 0) return;
    const uint8_t v = rc_comp(c);
    for (int64_t k = (int64_t)lo - 1; k >= 0 && hend[k] == hend[lo - 1]; --k) {
        if (i >= bend[k]) break;
        const uint32_t letters = let[bend[k]] - let[hend[k]];
        const uint32_t rank = let[i] - let[hend[k]];
        out[oo[nr - 1 - k] + (hend[k] - off[k]) + (letters - 1 - rank)] = v;
    }
}
