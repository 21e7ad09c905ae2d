"""forest_slam_amd — MI355X-native drop-in for the stereo-VO feature-correspondence path
of si220/Forest-SLAM (ros_ws/src/stereo_slam.py:84-306): ORB extraction, cross-checked
BF-Hamming matching, StereoSGBM-3way disparity, back-projection, PnP-RANSAC pose and a
windowed bundle adjustment, as hand-written HIP kernels for gfx950 behind a C ABI
(include/fvo.h).  See DESIGN.md."""
__version__ = "0.1.0"
