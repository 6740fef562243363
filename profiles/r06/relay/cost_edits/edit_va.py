import sys, os
p = os.path.join(sys.argv[1], "step_relay.h"); s = open(p).read()
a1 = """        listed = relay_list_read(r, epoch);
        ts[1] = relay_clock<ST>(listed);                            // its words published
        scalar_tail<KL>(p, b, lane, in, m);"""
b1 = """        scalar_tail<KL>(p, b, lane, in, m);
        listed = relay_list_read(r, epoch);
        ts[1] = relay_clock<ST>(listed);"""
a2 = """        listed = relay_list_read(r, epoch);
        ts[1] = relay_clock<ST>(listed);
        vec_tail<KL, KA, true>(p, b, lane, in, m);"""
b2 = """        vec_tail<KL, KA, true>(p, b, lane, in, m);
        listed = relay_list_read(r, epoch);
        ts[1] = relay_clock<ST>(listed);"""
for a, b in ((a1, b1), (a2, b2)):
    assert s.count(a) == 1, a
    s = s.replace(a, b)
open(p, "w").write(s)
