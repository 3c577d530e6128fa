"""Summary of tools/hptime_profile.py's stamps: per call the last publication,
the fit's end (last pair done), the HPDI's end, the items written after the
fit, the last items (their publication, take and write times), and the
publication-to-HPDI latency."""
import numpy as np
z = np.load('gpurun_out/hptime.npz')
T = int(z['T']); P = 30
for k in ('arr_0','arr_1','arr_2'):
    a = z[k].astype(np.int64)
    pub = a[:T]; pend = a[T:2*T]; take = a[2*T:2*T+T*P]; done = a[2*T+T*P:]
    t0 = pub[pub>0].min()
    f = lambda x: (x - t0) / 100.0  # us (100 MHz)
    fit_end = f(pend.max()); hp_end = f(done.max())
    print(f"{k}: first publish 0, last publish {f(pub.max()):.1f} us, fit end (last pair) {fit_end:.1f}, hpdi end {hp_end:.1f}; missing pub {(pub==0).sum()} pend {(pend==0).sum()} take {(take==0).sum()} done {(done==0).sum()}")
    # items done after the fit end
    late = done > pend.max()
    print(f"   items done after fit end: {late.sum()}  of taxa {len(np.unique(np.nonzero(late)[0]//P))}")
    idx = np.argsort(-done)[:12]
    for it in idx:
        t = it // P
        print(f"   item {it} taxon {t} pos {it%P}: pub {f(pub[t]):.1f} take {f(take[it]):.1f} done {f(done[it]):.1f} (proc {(done[it]-take[it])/100:.1f} us, wait {(take[it]-pub[t])/100:.1f}) pair-end {f(pend[t]):.1f}")
    # publish times of the last taxa
    lp = np.sort(f(pub))[-10:]
    print("   last publishes", np.round(lp,1))
    # per-taxon hpdi end - publish
    dtax = done.reshape(T,P).max(1)
    lat = (dtax - pub)/100
    print("   per-taxon hpdi latency after publish: median %.1f  p99 %.1f max %.1f us" % (np.median(lat), np.quantile(lat,.99), lat.max()))
    proc = (done - take)/100
    print("   item processing: median %.2f p99 %.1f max %.1f us" % (np.median(proc), np.quantile(proc,.99), proc.max()))
