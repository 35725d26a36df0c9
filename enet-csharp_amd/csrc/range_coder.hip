// range_coder.hip -- ENet's adaptive range coder over a batch of DGRAMs on
// gfx950: one DGRAM per lane, each lane with its own 4096-
// symbol model in HBM scratch.
// Reference: /root/reference/enet-csharp/ENet/c/compress.cs (constants :11-23,
// enet_symbol_rescale :52-67, enet_range_coder_compress :69-460,
// enet_range_coder_decompress :462-943); ENetSymbol layout include/compress.cs:7-24.
//
// The coder is adaptive and strictly sequential inside a DGRAM (every byte
// updates the model the next byte is coded with), so the only parallelism is
// across DGRAMs.  Each lane walks its own order-2 context trees: a chain of
// dependent 16-byte loads per byte, latency-bound, far from any HBM or VALU
// roofline.  The symbol rescale, recursive in the reference, is iterative here
// (an explicit stack of at most 256 frames: one per byte value on a left spine).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "range_coder.hpp"

namespace enethip {

namespace {

constexpr uint32_t kTop = 1u << 24, kBottom = 1u << 16;
constexpr uint32_t kCtxSymbolDelta = 3, kCtxSymbolMin = 1, kCtxEscapeMin = 1;
constexpr uint32_t kSubOrder = 2, kSubSymbolDelta = 2, kSubEscapeDelta = 5;

struct RSym {
    uint8_t value, count;
    uint16_t under, left, right, symbols, escapes, total, parent;
};
static_assert(sizeof(RSym) == 16, "ENetSymbol is 16 bytes");

struct Model {
    RSym* s;         // symbol 0 of this lane's kRangeSymbols
    uint32_t next;   // nextSymbol
    uint32_t stride; // symbols between this lane's consecutive symbols (1, or the lanes of the wave)
    __device__ __forceinline__ RSym& at(uint32_t i) const { return s[static_cast<size_t>(i) * stride]; }
};

__device__ __forceinline__ uint16_t add_symbol(Model& m, uint8_t value, uint8_t count) {
    const uint16_t i = static_cast<uint16_t>(m.next++);
    RSym y;
    y.value = value;
    y.count = count;
    y.under = count;
    y.left = y.right = y.symbols = y.escapes = y.total = y.parent = 0;
    m.at(i) = y;
    return i;
}

__device__ __forceinline__ uint16_t reset_model(Model& m) {
    m.next = 0;
    const uint16_t r = add_symbol(m, 0, 0);
    m.at(r).escapes = kCtxEscapeMin;
    m.at(r).total = static_cast<uint16_t>(kCtxEscapeMin + 256 * kCtxSymbolMin);
    return r;
}

// enet_symbol_rescale (compress.cs:52-67) without recursion: frame = the node
// whose left subtree is being rescaled and the running total of its chain.
__device__ uint16_t rescale_tree(Model& m, uint16_t i) {
    uint16_t st_node[256], st_total[256];
    int sp = 0;
    uint16_t total = 0;
    for (;;) {
        RSym& y = m.at(i);
        y.count = static_cast<uint8_t>(y.count - (y.count >> 1));
        y.under = y.count;
        if (y.left && sp < 256) {                           // descend: rescale the left subtree first
            st_node[sp] = i;
            st_total[sp] = total;
            ++sp;
            i = static_cast<uint16_t>(i + y.left);
            total = 0;
            continue;
        }
        for (;;) {                                          // node i done: add it, go right or return
            RSym& z = m.at(i);
            total = static_cast<uint16_t>(total + z.under);
            if (z.right) {
                i = static_cast<uint16_t>(i + z.right);
                break;
            }
            if (sp == 0) return total;
            --sp;                                           // a left subtree finished: its parent's under
            const uint16_t p = st_node[sp];
            m.at(p).under = static_cast<uint16_t>(m.at(p).under + total);
            total = st_total[sp];
            i = p;
        }
    }
}

__device__ __forceinline__ void rescale_context(Model& m, uint16_t ctx, uint32_t minimum) {
    RSym& x = m.at(ctx);
    const uint16_t t = x.symbols ? rescale_tree(m, static_cast<uint16_t>(ctx + x.symbols)) : 0;
    RSym& x2 = m.at(ctx);
    x2.escapes = static_cast<uint16_t>(x2.escapes - (x2.escapes >> 1));
    x2.total = static_cast<uint16_t>(t + x2.escapes + 256 * minimum);
}

// find-or-insert `value` in a context tree (ENET_CONTEXT_ENCODE / _ROOT_ENCODE)
__device__ uint16_t tree_encode(Model& m, uint16_t ctx, uint8_t value, uint16_t& under, uint16_t& count,
                                uint32_t delta, uint32_t minimum) {
    under = static_cast<uint16_t>(value * minimum);
    count = static_cast<uint16_t>(minimum);
    if (!m.at(ctx).symbols) {
        const uint16_t y = add_symbol(m, value, static_cast<uint8_t>(delta));
        m.at(ctx).symbols = static_cast<uint16_t>(y - ctx);
        return y;
    }
    uint16_t node = static_cast<uint16_t>(ctx + m.at(ctx).symbols);
    for (;;) {
        RSym n = m.at(node);
        if (value < n.value) {
            m.at(node).under = static_cast<uint16_t>(n.under + delta);
            if (n.left) {
                node = static_cast<uint16_t>(node + n.left);
                continue;
            }
            const uint16_t y = add_symbol(m, value, static_cast<uint8_t>(delta));
            m.at(node).left = static_cast<uint16_t>(y - node);
            return y;
        }
        if (value > n.value) {
            under = static_cast<uint16_t>(under + n.under);
            if (n.right) {
                node = static_cast<uint16_t>(node + n.right);
                continue;
            }
            const uint16_t y = add_symbol(m, value, static_cast<uint8_t>(delta));
            m.at(node).right = static_cast<uint16_t>(y - node);
            return y;
        }
        count = static_cast<uint16_t>(count + n.count);
        under = static_cast<uint16_t>(under + n.under - n.count);
        m.at(node).under = static_cast<uint16_t>(n.under + delta);
        m.at(node).count = static_cast<uint8_t>(n.count + delta);
        return node;
    }
}

// the decoder's search by cumulative frequency (ENET_CONTEXT_TRY_DECODE /
// _ROOT_DECODE); -1 = corrupt stream (the reference returns 0)
__device__ int tree_decode(Model& m, uint16_t ctx, uint16_t code, uint8_t& value, uint16_t& under, uint16_t& count,
                           uint32_t delta, uint32_t minimum, bool create) {
    under = 0;
    count = static_cast<uint16_t>(minimum);
    if (!m.at(ctx).symbols) {
        if (!create) return -1;
        value = static_cast<uint8_t>(code / minimum);
        under = static_cast<uint16_t>(code - code % minimum);
        const uint16_t y = add_symbol(m, value, static_cast<uint8_t>(delta));
        m.at(ctx).symbols = static_cast<uint16_t>(y - ctx);
        return y;
    }
    uint16_t node = static_cast<uint16_t>(ctx + m.at(ctx).symbols);
    for (;;) {
        RSym n = m.at(node);
        const uint16_t after = static_cast<uint16_t>(under + n.under + (n.value + 1) * minimum);
        const uint16_t before = static_cast<uint16_t>(n.count + minimum);
        if (code >= after) {
            under = static_cast<uint16_t>(under + n.under);
            if (n.right) {
                node = static_cast<uint16_t>(node + n.right);
                continue;
            }
            if (!create) return -1;
            value = static_cast<uint8_t>(n.value + 1 + (code - after) / minimum);
            under = static_cast<uint16_t>(code - (code - after) % minimum);
            const uint16_t y = add_symbol(m, value, static_cast<uint8_t>(delta));
            m.at(node).right = static_cast<uint16_t>(y - node);
            return y;
        }
        if (static_cast<int>(code) < static_cast<int>(after) - static_cast<int>(before)) {
            m.at(node).under = static_cast<uint16_t>(n.under + delta);
            if (n.left) {
                node = static_cast<uint16_t>(node + n.left);
                continue;
            }
            if (!create) return -1;
            const int gap = static_cast<int>(after) - static_cast<int>(before) - static_cast<int>(code) - 1;
            value = static_cast<uint8_t>(n.value - 1 - gap / static_cast<int>(minimum));
            under = static_cast<uint16_t>(code - gap % static_cast<int>(minimum));
            const uint16_t y = add_symbol(m, value, static_cast<uint8_t>(delta));
            m.at(node).left = static_cast<uint16_t>(y - node);
            return y;
        }
        value = n.value;
        count = static_cast<uint16_t>(count + n.count);
        under = static_cast<uint16_t>(after - before);
        m.at(node).under = static_cast<uint16_t>(n.under + delta);
        m.at(node).count = static_cast<uint8_t>(n.count + delta);
        return node;
    }
}

struct Encoder {
    uint32_t low = 0, range = ~0u;
    uint8_t* out;
    uint8_t* end;
    bool fail = false;
    __device__ void put(uint32_t under, uint32_t count, uint32_t total) {   // ENET_RANGE_CODER_ENCODE
        range /= total;
        low += under * range;
        range *= count;
        for (;;) {
            if ((low ^ (low + range)) >= kTop) {
                if (range >= kBottom) break;
                range = (0u - low) & (kBottom - 1);
            }
            if (out >= end) {
                fail = true;
                return;
            }
            *out++ = static_cast<uint8_t>(low >> 24);
            range <<= 8;
            low <<= 8;
        }
    }
};

// enet_range_coder_compress (compress.cs:69-460); 0 = does not fit
__device__ uint32_t compress_one(Model& m, const uint8_t* in, uint32_t n, uint8_t* out, uint32_t limit) {
    if (n == 0) return 0;
    Encoder e;
    e.out = out;
    e.end = out + limit;
    uint16_t root = reset_model(m);
    uint16_t predicted = 0;
    uint32_t order = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const uint8_t value = in[k];
        int parent = -1;                                    // -1: `predicted`, else that symbol's parent field
        uint16_t under, count, total, sym;
        bool coded = false;
        for (uint16_t sub = predicted; sub != root;) {
            sym = tree_encode(m, sub, value, under, count, kSubSymbolDelta, 0);
            if (parent < 0) predicted = sym;
            else m.at(parent).parent = sym;
            parent = sym;
            RSym& x = m.at(sub);
            total = x.total;
            if (count > 0) {
                e.put(static_cast<uint32_t>(x.escapes) + under, count, total);
            } else {
                if (x.escapes > 0 && x.escapes < total) e.put(0, x.escapes, total);
                x.escapes = static_cast<uint16_t>(x.escapes + kSubEscapeDelta);
                x.total = static_cast<uint16_t>(x.total + kSubEscapeDelta);
            }
            if (e.fail) return 0;
            x.total = static_cast<uint16_t>(x.total + kSubSymbolDelta);
            if (count > 0xFF - 2 * kSubSymbolDelta || x.total > kBottom - 0x100) rescale_context(m, sub, 0);
            if (count > 0) {
                coded = true;
                break;
            }
            sub = m.at(sub).parent;
        }
        if (!coded) {
            sym = tree_encode(m, root, value, under, count, kCtxSymbolDelta, kCtxSymbolMin);
            if (parent < 0) predicted = sym;
            else m.at(parent).parent = sym;
            RSym& r = m.at(root);
            e.put(static_cast<uint32_t>(r.escapes) + under, count, r.total);
            if (e.fail) return 0;
            r.total = static_cast<uint16_t>(r.total + kCtxSymbolDelta);
            if (count > 0xFF - 2 * kCtxSymbolDelta + kCtxSymbolMin || r.total > kBottom - 0x100)
                rescale_context(m, root, kCtxSymbolMin);
        }
        if (order >= kSubOrder) predicted = m.at(predicted).parent;   // nextInput (411-443)
        else ++order;
        if (m.next >= kRangeSymbols - kSubOrder) {
            root = reset_model(m);
            predicted = 0;
            order = 0;
        }
    }
    while (e.low) {                                          // flush (446-456)
        if (e.out >= e.end) return 0;
        *e.out++ = static_cast<uint8_t>(e.low >> 24);
        e.low <<= 8;
    }
    return static_cast<uint32_t>(e.out - out);
}

struct Decoder {
    uint32_t low = 0, code = 0, range = ~0u;
    const uint8_t* in;
    const uint8_t* end;
    __device__ void update(uint32_t under, uint32_t count) {   // ENET_RANGE_CODER_DECODE's update
        low += under * range;
        range *= count;
        for (;;) {
            if ((low ^ (low + range)) >= kTop) {
                if (range >= kBottom) break;
                range = (0u - low) & (kBottom - 1);
            }
            code <<= 8;
            if (in < end) code |= *in++;
            range <<= 8;
            low <<= 8;
        }
    }
};

// enet_range_coder_decompress (compress.cs:462-943); 0 = corrupt or does not fit
__device__ uint32_t decompress_one(Model& m, const uint8_t* in, uint32_t n, uint8_t* out, uint32_t limit) {
    if (n == 0) return 0;
    uint8_t* o = out;
    uint8_t* const oend = out + limit;
    Decoder d;
    d.in = in;
    d.end = in + n;
    uint16_t root = reset_model(m);
    uint16_t predicted = 0;
    uint32_t order = 0;
    for (int b = 24; b >= 0; b -= 8)
        if (d.in < d.end) d.code |= static_cast<uint32_t>(*d.in++) << b;
    for (;;) {
        uint8_t value = 0;
        uint16_t code, under, count, bottom = 0;
        int parent = -1;
        uint16_t sub = predicted;
        bool found = false;
        for (; sub != root; sub = m.at(sub).parent) {
            const RSym x = m.at(sub);
            if (x.escapes <= 0) continue;
            const uint16_t total = x.total;
            if (x.escapes >= total) continue;
            code = static_cast<uint16_t>((d.code - d.low) / (d.range /= total));
            if (code < x.escapes) {
                d.update(0, x.escapes);
                continue;
            }
            code = static_cast<uint16_t>(code - x.escapes);
            const int sym = tree_decode(m, sub, code, value, under, count, kSubSymbolDelta, 0, false);
            if (sym < 0) return 0;
            bottom = static_cast<uint16_t>(sym);
            RSym& xs = m.at(sub);
            d.update(static_cast<uint32_t>(xs.escapes) + under, count);
            xs.total = static_cast<uint16_t>(xs.total + kSubSymbolDelta);
            if (count > 0xFF - 2 * kSubSymbolDelta || xs.total > kBottom - 0x100) rescale_context(m, sub, 0);
            found = true;
            break;
        }
        if (!found) {
            const RSym r = m.at(root);
            code = static_cast<uint16_t>((d.code - d.low) / (d.range /= r.total));
            if (code < r.escapes) {
                d.update(0, r.escapes);
                break;                                       // end of stream (629-650)
            }
            code = static_cast<uint16_t>(code - r.escapes);
            bottom = static_cast<uint16_t>(
                tree_decode(m, root, code, value, under, count, kCtxSymbolDelta, kCtxSymbolMin, true));
            RSym& rr = m.at(root);
            d.update(static_cast<uint32_t>(rr.escapes) + under, count);
            rr.total = static_cast<uint16_t>(rr.total + kCtxSymbolDelta);
            if (count > 0xFF - 2 * kCtxSymbolDelta + kCtxSymbolMin || rr.total > kBottom - 0x100)
                rescale_context(m, root, kCtxSymbolMin);
            sub = root;
        }
        // patchContexts (789-898): the contexts passed over learn `value`
        for (uint16_t patch = predicted; patch != sub; patch = m.at(patch).parent) {
            uint16_t pu, pc;
            const uint16_t y = tree_encode(m, patch, value, pu, pc, kSubSymbolDelta, 0);
            if (parent < 0) predicted = y;
            else m.at(parent).parent = y;
            parent = y;
            RSym& p = m.at(patch);
            if (pc <= 0) {
                p.escapes = static_cast<uint16_t>(p.escapes + kSubEscapeDelta);
                p.total = static_cast<uint16_t>(p.total + kSubEscapeDelta);
            }
            p.total = static_cast<uint16_t>(p.total + kSubSymbolDelta);
            if (pc > 0xFF - 2 * kSubSymbolDelta || p.total > kBottom - 0x100) rescale_context(m, patch, 0);
        }
        if (parent < 0) predicted = bottom;
        else m.at(parent).parent = bottom;
        if (o >= oend) return 0;
        *o++ = value;
        if (order >= kSubOrder) predicted = m.at(predicted).parent;
        else ++order;
        if (m.next >= kRangeSymbols - kSubOrder) {
            root = reset_model(m);
            predicted = 0;
            order = 0;
        }
    }
    return static_cast<uint32_t>(o - out);
}

// `lanes` active lanes per wave: a wave runs its lanes' byte loops in lock step, so a
// byte costs the wave its slowest lane's tree walk; fewer lanes per wave (more waves)
// wait on fewer stragglers.
template <bool DECOMPRESS>
__global__ void __launch_bounds__(64) range_coder_kernel(RangeArgs a, uint32_t lanes) {
    if (threadIdx.x >= lanes) return;
    const uint64_t t = static_cast<uint64_t>(blockIdx.x) * lanes + threadIdx.x;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * lanes;
    Model m;
    // the wave's models: lane-major (each lane's symbols contiguous) or symbol-major
    // (symbol i of the wave's lanes side by side: the lanes' recent symbols share lines)
    RSym* const sc = reinterpret_cast<RSym*>(a.scratch);
    m.s = a.interleave ? sc + static_cast<uint64_t>(blockIdx.x) * lanes * kRangeSymbols + threadIdx.x
                       : sc + t * kRangeSymbols;
    m.stride = a.interleave ? lanes : 1u;
    m.next = 0;
    for (uint64_t i = t; i < a.n; i += stride) {
        const uint8_t* in = a.in + a.in_off[i];
        uint8_t* out = a.out + a.out_off[i];
        a.out_len[i] = DECOMPRESS ? decompress_one(m, in, a.in_len[i], out, a.out_limit[i])
                                  : compress_one(m, in, a.in_len[i], out, a.out_limit[i]);
    }
}

}  // namespace

int range_coder_launch(bool decompress, const RangeArgs& a, uint64_t threads, uint32_t lanes, hipStream_t st) {
    if (a.n == 0) return 0;
    if (lanes == 0 || lanes > 64) return -static_cast<int>(hipErrorInvalidValue);
    const unsigned grid =
        static_cast<unsigned>(std::max<uint64_t>(1, (std::min<uint64_t>(threads, a.n) + lanes - 1) / lanes));
    if (decompress) hipLaunchKernelGGL(range_coder_kernel<true>, dim3(grid), dim3(64), 0, st, a, lanes);
    else hipLaunchKernelGGL(range_coder_kernel<false>, dim3(grid), dim3(64), 0, st, a, lanes);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -static_cast<int>(e);
}

}  // namespace enethip
