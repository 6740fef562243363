import sys, os
p = os.path.join(sys.argv[1], "env_step.h"); s = open(p).read()
old1 = "        o[e] = pick(!shift_w && f == F - 1, un[e], sh[e]);"
new1 = "        o[e] = pick(!shift_w & (f == F - 1), un[e], sh[e]);"
old2 = "    if (kk + 3 >= WF - F || (!shift_w && (uint32_t)(slot_w - kk) <= 3u)) {   // a last day or the slot"
new2 = "    if ((kk + 3 >= WF - F) | (!shift_w & ((uint32_t)(slot_w - kk) <= 3u))) {   // a last day or the slot"
old3 = """            const bool in_row = pos < WF;
            const bool lastday = in_row && pos >= WF - F;
            const float bsel = pick(f == 0, xb.x, pick(f == 1, xb.y, pick(f == 2, xb.z, xb.w)));
            o[e] = pick(lastday && f < F - 1, bsel, o[e]);
            o[e] = pick(shift_w ? (lastday && f == F - 1) : (in_row && pos == slot_w), xwp, o[e]);"""
new3 = """            const bool in_row = pos < WF;
            const bool lastday = in_row & (pos >= WF - F);
            const float bsel = pick(f == 0, xb.x, pick(f == 1, xb.y, pick(f == 2, xb.z, xb.w)));
            o[e] = pick(lastday & (f < F - 1), bsel, o[e]);
            o[e] = pick((shift_w & lastday & (f == F - 1)) | (!shift_w & in_row & (pos == slot_w)), xwp, o[e]);"""
for a, b in ((old1, new1), (old2, new2), (old3, new3)):
    assert s.count(a) == 1, a
    s = s.replace(a, b)
open(p, "w").write(s)
