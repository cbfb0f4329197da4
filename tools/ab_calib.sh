for r in 1 2; do for lib in "" yet-another-halo2-fork_amd/lib_ab/libh2g_sp1all.so; do
H2G_LIB=$lib timeout -k 10 60 python3 -c "
import sys; sys.path.insert(0,'yet-another-halo2-fork_amd'); import h2g; h2g.init([0]); c=h2g.box_calibrate(); print('$lib'[-12:], round(c['modmul_f29_gps'],1), round(c['modmul_fips2_gps'],1), round(c['sclk_ghz_in_kernel'],3))" || exit 1
done; done
