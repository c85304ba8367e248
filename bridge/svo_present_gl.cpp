// svo_present_gl.cpp — the shim's frame on screen: the replacement of render()'s draw of the low_res program
// (src/main.cpp:73 glUseProgram(lowResProgram), :105-107 glBindVertexArray / glBindBuffer / glDrawArrays).
//
// svoPresentShaded(width, height, time) renders the shaded frame (svoRenderShaded: pick ray for lookingAtBlock,
// primary rays, shadow rays, reflections, refraction through the scene) straight into a GL pixel-unpack buffer that
// HIP has registered (hip_gl_interop.h), so the image never leaves the GPU: map -> svoRenderShaded into the mapped
// pointer -> unmap on the same stream (GL commands issued after the unmap see the finished image) -> glTexSubImage2D
// from that buffer into an RGBA32F texture -> glBlitFramebuffer of the texture onto the default framebuffer.
// Pixel k of the image is (k % width, k / width) with rows counted from the bottom, as gl_FragCoord counts them
// (low_res.frag:264-265), which is also a GL texture's row order: no flip.
//
// Needs the application's current GL context (GL 3.0: buffer and framebuffer objects, glBlitFramebuffer), which the
// reference creates in createWindow / setupOpenGl (src/setup.cpp:55-447) before render() runs.  In the reference build
// the GL entry points come from GLEW (src/globals.hpp includes <GL/glew.h>); elsewhere (this repository's compile
// check, tests/test_bridge_link.py) from the system's <GL/gl.h> + <GL/glext.h> prototypes.
#if __has_include(<GL/glew.h>)
#include <GL/glew.h>
#else
#define GL_GLEXT_PROTOTYPES 1
#include <GL/gl.h>
#include <GL/glext.h>
#endif
#include <hip/hip_runtime_api.h>  // (before hip_gl_interop.h, which uses its types)
#include <hip/hip_gl_interop.h>
#include <stdio.h>
#include <stdlib.h>

#include "svo_bridge.hpp"

namespace {

struct Present {
    int32_t w = 0, h = 0;
    GLuint pbo = 0, tex = 0, fbo = 0;
    hipGraphicsResource_t res = nullptr;
};
Present g_present;

void fail(const char* what, int code) {
    fprintf(stderr, "svo_bridge: svoPresentShaded: %s failed (%d)\n", what, code);
    exit(1);  // (the reference's own failure convention for GL errors, src/globals.hpp:32-43)
}

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) fail(what, (int)e);
}

void release(Present& p) {
    if (p.res) hip_ok(hipGraphicsUnregisterResource(p.res), "hipGraphicsUnregisterResource");
    if (p.fbo) glDeleteFramebuffers(1, &p.fbo);
    if (p.tex) glDeleteTextures(1, &p.tex);
    if (p.pbo) glDeleteBuffers(1, &p.pbo);
    p = Present{};
}

// the frame's buffer (width * height float4), texture and read framebuffer, (re)made when the size changes
// (main.cpp's dimensionsChanged)
void ensure(Present& p, int32_t width, int32_t height) {
    if (p.pbo && p.w == width && p.h == height) return;
    release(p);
    p.w = width;
    p.h = height;
    glGenBuffers(1, &p.pbo);
    glBindBuffer(GL_PIXEL_UNPACK_BUFFER, p.pbo);
    glBufferData(GL_PIXEL_UNPACK_BUFFER, (GLsizeiptr)width * height * 4 * sizeof(float), nullptr, GL_STREAM_DRAW);
    glBindBuffer(GL_PIXEL_UNPACK_BUFFER, 0);
    // HIP writes it and never reads it
    hip_ok(hipGraphicsGLRegisterBuffer(&p.res, p.pbo, hipGraphicsRegisterFlagsWriteDiscard), "hipGraphicsGLRegisterBuffer");
    glGenTextures(1, &p.tex);
    glBindTexture(GL_TEXTURE_2D, p.tex);
    glTexImage2D(GL_TEXTURE_2D, 0, GL_RGBA32F, width, height, 0, GL_RGBA, GL_FLOAT, nullptr);
    glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MIN_FILTER, GL_NEAREST);
    glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MAG_FILTER, GL_NEAREST);
    glBindTexture(GL_TEXTURE_2D, 0);
    glGenFramebuffers(1, &p.fbo);
    glBindFramebuffer(GL_READ_FRAMEBUFFER, p.fbo);
    glFramebufferTexture2D(GL_READ_FRAMEBUFFER, GL_COLOR_ATTACHMENT0, GL_TEXTURE_2D, p.tex, 0);
    const GLenum st = glCheckFramebufferStatus(GL_READ_FRAMEBUFFER);
    glBindFramebuffer(GL_READ_FRAMEBUFFER, 0);
    if (st != GL_FRAMEBUFFER_COMPLETE) fail("glCheckFramebufferStatus", (int)st);
}

}  // namespace

void svoPresentShaded(int32_t width, int32_t height, float time, hipStream_t stream) {
    Present& p = g_present;
    ensure(p, width, height);
    hip_ok(hipGraphicsMapResources(1, &p.res, stream), "hipGraphicsMapResources");
    void* img = nullptr;
    size_t bytes = 0;
    hip_ok(hipGraphicsResourceGetMappedPointer(&img, &bytes, p.res), "hipGraphicsResourceGetMappedPointer");
    if (bytes < (size_t)width * height * 4 * sizeof(float)) fail("mapped buffer size", (int)bytes);
    svoRenderShaded(width, height, static_cast<float*>(img), stream, time);
    hip_ok(hipGraphicsUnmapResources(1, &p.res, stream), "hipGraphicsUnmapResources");
    glBindBuffer(GL_PIXEL_UNPACK_BUFFER, p.pbo);
    glBindTexture(GL_TEXTURE_2D, p.tex);
    glTexSubImage2D(GL_TEXTURE_2D, 0, 0, 0, width, height, GL_RGBA, GL_FLOAT, nullptr);  // (from the bound buffer)
    glBindTexture(GL_TEXTURE_2D, 0);
    glBindBuffer(GL_PIXEL_UNPACK_BUFFER, 0);
    glBindFramebuffer(GL_READ_FRAMEBUFFER, p.fbo);
    glBindFramebuffer(GL_DRAW_FRAMEBUFFER, 0);
    glBlitFramebuffer(0, 0, width, height, 0, 0, width, height, GL_COLOR_BUFFER_BIT, GL_NEAREST);
    glBindFramebuffer(GL_READ_FRAMEBUFFER, 0);
}

void svoPresentRelease() { release(g_present); }
