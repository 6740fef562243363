import sys, os
p = os.path.join(sys.argv[1], "step_relay.h"); s = open(p).read()
a = """    const uint64_t lw = relay_get(r.list);
    return (uint32_t)(lw >> 32) == epoch ? (uint32_t)lw : 0u;
}"""
b = """    return 0u;                                   // probe: the block reads the list once (relay_adopt)
}"""
assert s.count(a) == 1; s = s.replace(a, b)
a = """    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sh_ok[wave] = (int32_t)__builtin_amdgcn_readfirstlane(listed);
    __syncthreads();
    uint32_t n = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / 64; ++w) n = max(n, (uint32_t)sh_ok[w]);
    if (n == 0) return;
    const KArgs ka = kargs();
    const RelayCtx c = relay_ctx<SEQ>(ka.r);"""
b = """    (void)listed;
    __syncthreads();                             // every wave's words completed (relay_list_read's wait)
    const KArgs ka = kargs();
    const RelayCtx c = relay_ctx<SEQ>(ka.r);
    if (threadIdx.x == 0) {
        const uint64_t lw = relay_get(ka.r.list);
        sh_ok[kB] = (uint32_t)(lw >> 32) == c.epoch ? (int32_t)(uint32_t)lw : 0;
    }
    __syncthreads();
    const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane(sh_ok[kB]);
    if (n == 0) return;"""
assert s.count(a) == 1, "adopt"; s = s.replace(a, b)
open(p, "w").write(s)
