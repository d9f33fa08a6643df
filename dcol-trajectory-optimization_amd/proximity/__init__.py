"""Drop-in for the reference's ``proximity`` package (proximity/proximity.py,
proximity/proximity_gradient.py).  Same import paths and signatures; every solve runs in
the HIP kernels of lib/libdcol.so."""
