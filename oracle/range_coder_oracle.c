/*
 * range_coder_oracle.c -- CPU ORACLE for ENet's adaptive range coder
 * (SURVEY.md 8f row 4).  TEST INFRASTRUCTURE ONLY: loaded by tests/ as the
 * checker of the batched GPU coder, never linked into libenethip.
 *
 * Plain-C restatement of /root/reference/enet-csharp/ENet/c/compress.cs:
 *   :11-23    constants (TOP 2^24, BOTTOM 2^16, context / subcontext deltas, order 2)
 *   :52-67    enet_symbol_rescale (recursive, as the reference)
 *   :69-460   enet_range_coder_compress
 *   :462-943  enet_range_coder_decompress
 * with the symbol layout of include/compress.cs:7-24 (16-byte ENetSymbol, 4096 of
 * them per coder).  The reference's macros are restated as small functions; the
 * arithmetic (16-bit counters, 8-bit counts, 32-bit coder state, wraparound) is
 * kept exactly.  Parity pinning: the reference tests never enable compression
 * and the C# cannot run here, so beyond this line-by-line restatement the pin is
 * the round trip decompress(compress(x)) == x on every test input
 * (tests/test_range_coder.py); exact compressed bytes are "parity unpinned"
 * against the reference itself.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define RC_TOP (1u << 24)
#define RC_BOTTOM (1u << 16)
#define CTX_SYMBOL_DELTA 3u
#define CTX_SYMBOL_MIN 1u
#define CTX_ESCAPE_MIN 1u
#define SUB_ORDER 2u
#define SUB_SYMBOL_DELTA 2u
#define SUB_ESCAPE_DELTA 5u
#define NSYM 4096u

typedef struct {
    uint8_t value, count;
    uint16_t under, left, right, symbols, escapes, total, parent;
} Sym;

typedef struct {
    Sym s[NSYM];
    uint32_t next;
} Coder;

static uint16_t new_symbol(Coder* c, uint8_t value, uint8_t count) {
    uint16_t i = (uint16_t)c->next++;
    Sym* y = &c->s[i];
    y->value = value;
    y->count = count;
    y->under = count;
    y->left = y->right = y->symbols = y->escapes = y->total = y->parent = 0;
    return i;
}

static uint16_t new_root(Coder* c) {
    c->next = 0;
    uint16_t r = new_symbol(c, 0, 0);
    c->s[r].escapes = CTX_ESCAPE_MIN;
    c->s[r].total = (uint16_t)(CTX_ESCAPE_MIN + 256 * CTX_SYMBOL_MIN);
    return r;
}

/* compress.cs:52-67 */
static uint16_t rescale(Coder* c, uint16_t i) {
    uint16_t total = 0;
    for (;;) {
        Sym* y = &c->s[i];
        y->count = (uint8_t)(y->count - (y->count >> 1));
        y->under = y->count;
        if (y->left) y->under = (uint16_t)(y->under + rescale(c, (uint16_t)(i + y->left)));
        total = (uint16_t)(total + y->under);
        if (!y->right) break;
        i = (uint16_t)(i + y->right);
    }
    return total;
}

/* the context rescale after an update (compress.cs:277-282 and their copies);
 * minimum = CTX_SYMBOL_MIN for the root context, 0 for subcontexts */
static void context_rescale(Coder* c, uint16_t ctx, uint32_t minimum) {
    Sym* x = &c->s[ctx];
    x->total = x->symbols ? rescale(c, (uint16_t)(ctx + x->symbols)) : 0;
    x->escapes = (uint16_t)(x->escapes - (x->escapes >> 1));
    x->total = (uint16_t)(x->total + x->escapes + 256 * minimum);
}

/* ENET_CONTEXT_ENCODE / _ROOT_ENCODE's symbol search (compress.cs:126-215 /
 * 288-373): find or insert `value` in the context's tree; *under / *count get the
 * cumulative frequency below it and its count (0 if it was just inserted). */
static uint16_t context_encode(Coder* c, uint16_t ctx, uint8_t value, uint16_t* under, uint16_t* count,
                               uint32_t delta, uint32_t minimum) {
    *under = (uint16_t)(value * minimum);
    *count = (uint16_t)minimum;
    Sym* x = &c->s[ctx];
    if (!x->symbols) {
        uint16_t y = new_symbol(c, value, (uint8_t)delta);
        c->s[ctx].symbols = (uint16_t)(y - ctx);
        return y;
    }
    uint16_t node = (uint16_t)(ctx + x->symbols);
    for (;;) {
        Sym* n = &c->s[node];
        if (value < n->value) {
            n->under = (uint16_t)(n->under + delta);
            if (n->left) { node = (uint16_t)(node + n->left); continue; }
            uint16_t y = new_symbol(c, value, (uint8_t)delta);
            c->s[node].left = (uint16_t)(y - node);
            return y;
        } else if (value > n->value) {
            *under = (uint16_t)(*under + n->under);
            if (n->right) { node = (uint16_t)(node + n->right); continue; }
            uint16_t y = new_symbol(c, value, (uint8_t)delta);
            c->s[node].right = (uint16_t)(y - node);
            return y;
        } else {
            *count = (uint16_t)(*count + n->count);
            *under = (uint16_t)(*under + n->under - n->count);
            n->under = (uint16_t)(n->under + delta);
            n->count = (uint8_t)(n->count + delta);
            return node;
        }
    }
}

typedef struct {
    uint32_t low, range;
    uint8_t *out, *end;
    int fail;
} Enc;

/* ENET_RANGE_CODER_ENCODE (compress.cs:224-242) */
static void encode(Enc* e, uint32_t under, uint32_t count, uint32_t total) {
    e->range /= total;
    e->low += under * e->range;
    e->range *= count;
    for (;;) {
        if ((e->low ^ (e->low + e->range)) >= RC_TOP) {
            if (e->range >= RC_BOTTOM) break;
            e->range = (uint32_t)(-e->low) & (RC_BOTTOM - 1);
        }
        if (e->out >= e->end) { e->fail = 1; return; }
        *e->out++ = (uint8_t)(e->low >> 24);
        e->range <<= 8;
        e->low <<= 8;
    }
}

/* compress.cs:69-460.  in[0..n) is the DGRAM (the reference's buffer list,
 * concatenated).  Returns the compressed size, 0 if it does not fit outLimit. */
size_t oracle_range_compress(const uint8_t* in, size_t n, uint8_t* out, size_t outLimit) {
    static __thread Coder coder;
    Coder* c = &coder;
    if (n == 0) return 0;
    Enc e = {0, ~0u, out, out + outLimit, 0};
    uint16_t root = new_root(c);
    uint16_t predicted = 0;
    uint32_t order = 0;
    for (size_t k = 0; k < n; ++k) {
        const uint8_t value = in[k];
        int parent = -1;                       /* -1: the `predicted` variable, else that symbol's parent field */
        uint16_t under, count, total, sym;
        int done = 0;
        uint16_t sub = predicted;
        while (sub != root) {
            sym = context_encode(c, sub, value, &under, &count, SUB_SYMBOL_DELTA, 0);
            if (parent < 0) predicted = sym; else c->s[parent].parent = sym;
            parent = sym;
            total = c->s[sub].total;
            if (count > 0) {
                encode(&e, (uint32_t)c->s[sub].escapes + under, count, total);
            } else {
                if (c->s[sub].escapes > 0 && c->s[sub].escapes < total) encode(&e, 0, c->s[sub].escapes, total);
                c->s[sub].escapes = (uint16_t)(c->s[sub].escapes + SUB_ESCAPE_DELTA);
                c->s[sub].total = (uint16_t)(c->s[sub].total + SUB_ESCAPE_DELTA);
            }
            if (e.fail) return 0;
            c->s[sub].total = (uint16_t)(c->s[sub].total + SUB_SYMBOL_DELTA);
            if (count > 0xFF - 2 * SUB_SYMBOL_DELTA || c->s[sub].total > RC_BOTTOM - 0x100) context_rescale(c, sub, 0);
            if (count > 0) { done = 1; break; }
            sub = c->s[sub].parent;
        }
        if (!done) {
            sym = context_encode(c, root, value, &under, &count, CTX_SYMBOL_DELTA, CTX_SYMBOL_MIN);
            if (parent < 0) predicted = sym; else c->s[parent].parent = sym;
            total = c->s[root].total;
            encode(&e, (uint32_t)c->s[root].escapes + under, count, total);
            if (e.fail) return 0;
            c->s[root].total = (uint16_t)(c->s[root].total + CTX_SYMBOL_DELTA);
            if (count > 0xFF - 2 * CTX_SYMBOL_DELTA + CTX_SYMBOL_MIN || c->s[root].total > RC_BOTTOM - 0x100)
                context_rescale(c, root, CTX_SYMBOL_MIN);
        }
        /* nextInput (compress.cs:411-443) */
        if (order >= SUB_ORDER) predicted = c->s[predicted].parent;
        else order++;
        if (c->next >= NSYM - SUB_ORDER) {
            root = new_root(c);
            predicted = 0;
            order = 0;
        }
    }
    while (e.low) {                            /* ENET_RANGE_CODER_FLUSH (446-456) */
        if (e.out >= e.end) return 0;
        *e.out++ = (uint8_t)(e.low >> 24);
        e.low <<= 8;
    }
    return (size_t)(e.out - out);
}

typedef struct {
    uint32_t low, code, range;
    const uint8_t *in, *end;
} Dec;

static void decode_update(Dec* d, uint32_t under, uint32_t count) {
    d->low += under * d->range;
    d->range *= count;
    for (;;) {
        if ((d->low ^ (d->low + d->range)) >= RC_TOP) {
            if (d->range >= RC_BOTTOM) break;
            d->range = (uint32_t)(-d->low) & (RC_BOTTOM - 1);
        }
        d->code <<= 8;
        if (d->in < d->end) d->code |= *d->in++;
        d->range <<= 8;
        d->low <<= 8;
    }
}

/* ENET_CONTEXT_DECODE's search in a context tree (compress.cs:543-595 for
 * subcontexts, 653-759 for the root): returns the symbol index, or -1 where the
 * reference returns 0 (a corrupt stream). */
static int context_decode(Coder* c, uint16_t ctx, uint16_t code, uint8_t* value, uint16_t* under, uint16_t* count,
                          uint32_t delta, uint32_t minimum, int create) {
    *under = 0;
    *count = (uint16_t)minimum;
    Sym* x = &c->s[ctx];
    if (!x->symbols) {
        if (!create) return -1;
        *value = (uint8_t)(code / minimum);
        *under = (uint16_t)(code - code % minimum);
        uint16_t y = new_symbol(c, *value, (uint8_t)delta);
        c->s[ctx].symbols = (uint16_t)(y - ctx);
        return y;
    }
    uint16_t node = (uint16_t)(ctx + x->symbols);
    for (;;) {
        Sym* n = &c->s[node];
        uint16_t after = (uint16_t)(*under + n->under + (n->value + 1) * minimum);
        uint16_t before = (uint16_t)(n->count + minimum);
        if (code >= after) {
            *under = (uint16_t)(*under + n->under);
            if (n->right) { node = (uint16_t)(node + n->right); continue; }
            if (!create) return -1;
            *value = (uint8_t)(n->value + 1 + (code - after) / minimum);
            *under = (uint16_t)(code - (code - after) % minimum);
            uint16_t y = new_symbol(c, *value, (uint8_t)delta);
            c->s[node].right = (uint16_t)(y - node);
            return y;
        } else if ((int)code < (int)after - (int)before) {         /* int arithmetic, as the C# */
            n->under = (uint16_t)(n->under + delta);
            if (n->left) { node = (uint16_t)(node + n->left); continue; }
            if (!create) return -1;
            const int gap = (int)after - (int)before - (int)code - 1;
            *value = (uint8_t)(n->value - 1 - gap / (int)minimum);
            *under = (uint16_t)(code - gap % (int)minimum);
            uint16_t y = new_symbol(c, *value, (uint8_t)delta);
            c->s[node].left = (uint16_t)(y - node);
            return y;
        } else {
            *value = n->value;
            *count = (uint16_t)(*count + n->count);
            *under = (uint16_t)(after - before);
            n->under = (uint16_t)(n->under + delta);
            n->count = (uint8_t)(n->count + delta);
            return node;
        }
    }
}

/* compress.cs:462-943.  Returns the decompressed size, 0 on a corrupt stream or
 * when the output does not fit outLimit. */
size_t oracle_range_decompress(const uint8_t* in, size_t inLimit, uint8_t* out, size_t outLimit) {
    static __thread Coder coder;
    Coder* c = &coder;
    if (inLimit == 0) return 0;
    uint8_t* o = out;
    uint8_t* oend = out + outLimit;
    Dec d = {0, 0, ~0u, in, in + inLimit};
    uint16_t root = new_root(c);
    uint16_t predicted = 0;
    uint32_t order = 0;
    for (int b = 24; b >= 0; b -= 8)
        if (d.in < d.end) d.code |= (uint32_t)(*d.in++) << b;
    for (;;) {
        uint8_t value = 0;
        uint16_t code, under, count, total, bottom;
        int parent = -1;
        int sym;
        uint16_t sub;
        int found = 0;
        for (sub = predicted; sub != root; sub = c->s[sub].parent) {
            Sym* x = &c->s[sub];
            if (x->escapes <= 0) continue;
            total = x->total;
            if (x->escapes >= total) continue;
            code = (uint16_t)((d.code - d.low) / (d.range /= total));
            if (code < x->escapes) {
                decode_update(&d, 0, x->escapes);
                continue;
            }
            code = (uint16_t)(code - x->escapes);
            sym = context_decode(c, sub, code, &value, &under, &count, SUB_SYMBOL_DELTA, 0, 0);
            if (sym < 0) return 0;
            bottom = (uint16_t)sym;
            decode_update(&d, (uint32_t)c->s[sub].escapes + under, count);
            c->s[sub].total = (uint16_t)(c->s[sub].total + SUB_SYMBOL_DELTA);
            if (count > 0xFF - 2 * SUB_SYMBOL_DELTA || c->s[sub].total > RC_BOTTOM - 0x100) context_rescale(c, sub, 0);
            found = 1;
            break;
        }
        if (!found) {
            total = c->s[root].total;
            code = (uint16_t)((d.code - d.low) / (d.range /= total));
            if (code < c->s[root].escapes) {
                decode_update(&d, 0, c->s[root].escapes);
                break;                          /* end of stream (compress.cs:629-650) */
            }
            code = (uint16_t)(code - c->s[root].escapes);
            sym = context_decode(c, root, code, &value, &under, &count, CTX_SYMBOL_DELTA, CTX_SYMBOL_MIN, 1);
            bottom = (uint16_t)sym;
            decode_update(&d, (uint32_t)c->s[root].escapes + under, count);
            c->s[root].total = (uint16_t)(c->s[root].total + CTX_SYMBOL_DELTA);
            if (count > 0xFF - 2 * CTX_SYMBOL_DELTA + CTX_SYMBOL_MIN || c->s[root].total > RC_BOTTOM - 0x100)
                context_rescale(c, root, CTX_SYMBOL_MIN);
            sub = root;
        }
        /* patchContexts (compress.cs:789-898): the contexts passed over learn `value` */
        for (uint16_t patch = predicted; patch != sub; patch = c->s[patch].parent) {
            uint16_t pu, pc;
            uint16_t y = context_encode(c, patch, value, &pu, &pc, SUB_SYMBOL_DELTA, 0);
            if (parent < 0) predicted = y; else c->s[parent].parent = y;
            parent = y;
            if (pc <= 0) {
                c->s[patch].escapes = (uint16_t)(c->s[patch].escapes + SUB_ESCAPE_DELTA);
                c->s[patch].total = (uint16_t)(c->s[patch].total + SUB_ESCAPE_DELTA);
            }
            c->s[patch].total = (uint16_t)(c->s[patch].total + SUB_SYMBOL_DELTA);
            if (pc > 0xFF - 2 * SUB_SYMBOL_DELTA || c->s[patch].total > RC_BOTTOM - 0x100) context_rescale(c, patch, 0);
        }
        if (parent < 0) predicted = bottom; else c->s[parent].parent = bottom;
        if (o >= oend) return 0;
        *o++ = value;
        if (order >= SUB_ORDER) predicted = c->s[predicted].parent;
        else order++;
        if (c->next >= NSYM - SUB_ORDER) {
            root = new_root(c);
            predicted = 0;
            order = 0;
        }
    }
    return (size_t)(o - out);
}

/* Batches: DGRAM i is in[inOff[i] .. +inLen[i]), its output goes to
 * out[outOff[i] .. +outLimit[i]), its size (0 = did not fit / corrupt) to outLen[i]. */
void oracle_range_compress_batch(const uint8_t* in, const uint64_t* inOff, const uint32_t* inLen, size_t n,
                                 uint8_t* out, const uint64_t* outOff, const uint32_t* outLimit, uint32_t* outLen) {
    for (size_t i = 0; i < n; ++i)
        outLen[i] = (uint32_t)oracle_range_compress(in + inOff[i], inLen[i], out + outOff[i], outLimit[i]);
}

void oracle_range_decompress_batch(const uint8_t* in, const uint64_t* inOff, const uint32_t* inLen, size_t n,
                                   uint8_t* out, const uint64_t* outOff, const uint32_t* outLimit, uint32_t* outLen) {
    for (size_t i = 0; i < n; ++i)
        outLen[i] = (uint32_t)oracle_range_decompress(in + inOff[i], inLen[i], out + outOff[i], outLimit[i]);
}
