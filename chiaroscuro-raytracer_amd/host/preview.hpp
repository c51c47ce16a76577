// preview.hpp -- the render side of the interactive preview without a window
// (SURVEY §8f-4): OpenGLPreview's camera, R / TAB / = / - / WASDQE / mouse
// handling and Screen::requestRender / updateScreen (src/openglPreview.cpp:12-257,
// src/camera.cpp), driving the GPU RayTracer.  The GL drawing of the model and
// the window are out of scope (no GLFW here); what a frame shows after R is
// exactly RayTracer::getData() after normalizeImage(), as Screen::updateScreen
// uploads it as the screen texture.
#pragma once
#include "raytracer.hpp"

namespace chiaro {

enum CameraMovement { FORWARD, BACKWARD, LEFT, RIGHT, UPWARD, DOWNWARD }; // include/camera.hpp:13

// src/camera.cpp (LearnOpenGL camera as the reference modifies it), float members,
// the C library's double trigonometry as the unqualified calls there resolve.
struct PreviewCamera {
    vec3 Position, Front, Up, Right, WorldUp;
    float Yaw = -90.f, Pitch = 0.f, MovementSpeed = 2.5f, MouseSensitivity = 0.1f, Zoom = 90.f;
    PreviewCamera(vec3 position, vec3 lookAt, vec3 up);
    void ProcessKeyboard(CameraMovement direction, float deltaTime);
    void ProcessMouseMovement(float xoffset, float yoffset, bool constrainPitch = true);
    void ProcessMouseScroll(float yoffset);
    void updateCameraVectors();
};

// OpenGLPreview's initial Zoom: glm::degrees(2 * atanf(0.5 * yview)) (src/openglPreview.cpp:39)
float preview_zoom(float yview);

class PreviewSession {
  public:
    // OpenGLPreview(Scene*) + setRenderer: camera from VP / LA / UP, Zoom from yview
    PreviewSession(Scene &scene, RayTracer &renderer);
    // key R pressed (one render per press): Screen::requestRender -- a layer at the
    // camera (the RayTracer accumulates while the camera stays put), then updateScreen
    void pressRender();
    // keys = / -: exposure +- 0.2, re-normalise the last render (no new layer)
    void exposureUp();
    void exposureDown();
    void toggleView() { showRender = !showRender; } // TAB
    // WASDQE / mouse / scroll: ignored while the render is shown, as processInputs does
    void move(CameraMovement d, float deltaTime, bool fast = false);
    void shiftState(bool fast);
    void look(float xoffset, float yoffset);
    void scroll(float yoffset);
    // Screen::updateScreen: normalizeImage() with the scene's exposure, texture = getData()
    const uint8_t *updateScreen();
    const uint8_t *texture() { return renderer.getData(); }
    unsigned width() const { return scene.xres; }
    unsigned height() const { return scene.yres; }
    PreviewCamera camera;
    bool showRender = false;
    unsigned renders = 0;

  private:
    Scene &scene;
    RayTracer &renderer;
};

} // namespace chiaro
