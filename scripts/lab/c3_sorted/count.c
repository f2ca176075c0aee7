// snappy element count per record (lab helper for c3_sorted.py): stream at record + 12 + k
#include <stdint.h>
#include <string.h>
void count_elements(const uint8_t *src, const uint64_t *off, const uint32_t *len, uint32_t n, uint32_t *out) {
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t *r = src + off[i];
        uint32_t k;
        memcpy(&k, r, 4);
        const uint8_t *s = r + 12 + k, *e = r + len[i];
        while (s < e && (*s & 0x80)) s++;
        s++;
        uint32_t c = 0;
        while (s < e) {
            const uint32_t t = *s, ty = t & 3, x = t >> 2;
            if (ty == 0) {
                uint32_t ln;
                if (x < 60) { ln = x + 1; s += 1; }
                else { uint32_t nb = x - 59; ln = 0; memcpy(&ln, s + 1, nb); ln += 1; s += 1 + nb; }
                s += ln;
            } else s += ty == 1 ? 2 : ty == 2 ? 3 : 5;
            c++;
        }
        out[i] = c;
    }
}
