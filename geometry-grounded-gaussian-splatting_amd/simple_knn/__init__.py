"""MI355X drop-in for the reference's `simple_knn` extension
(submodules/simple-knn): `from simple_knn._C import distCUDA2`
(scene/gaussian_model.py:20) resolves here once this directory's parent is on
sys.path.  The compute is gsr_knn_mean_dist in libgsr.so (csrc/knn.hip);
there is no CPU fallback.
"""
