"""rtzig — MI355X-native drop-in for the per-pixel sampling hot path of
AndrewJarrett/raytracing-with-zig (Camera.render, src/camera.zig:123-145).

Product path: C ABI (include/rt.h) -> librtzig.so -> HIP megakernel on gfx950.
"""
from .abi import (RT_DIELECTRIC, RT_LAMBERTIAN, RT_METAL, RT_OUT_LINEAR_F64, RT_OUT_RGB8,
                  RtCamera, RtCameraParams, RtOptions, RtSphere)
from .api import (PPM, Camera, CameraBuilder, DeviceRenderer, Scene, chapter9_camera,
                  chapter13_camera, encode_p3, encode_p6, final_scene_camera, release_cached_contexts, render,
                  sample_key, to_rgb8)
from .lib import EXPORTED, LIB_PATH, RtError, load

__all__ = [
    "RT_DIELECTRIC", "RT_LAMBERTIAN", "RT_METAL", "RT_OUT_LINEAR_F64", "RT_OUT_RGB8",
    "RtCamera", "RtCameraParams", "RtOptions", "RtSphere",
    "PPM", "Camera", "CameraBuilder", "DeviceRenderer", "Scene", "chapter9_camera",
    "chapter13_camera", "encode_p3", "encode_p6", "final_scene_camera", "release_cached_contexts", "render",
    "sample_key", "to_rgb8",
    "EXPORTED", "LIB_PATH", "RtError", "load",
]
