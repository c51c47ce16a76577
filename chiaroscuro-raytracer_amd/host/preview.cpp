// preview.cpp -- headless counterpart of the preview's render path (preview.hpp).
#include "preview.hpp"

#include <math.h>

#include <iostream>

namespace chiaro {

namespace {
// glm::radians / glm::degrees on float (gtc/constants, func_trigonometric.inl)
float radians(float d) { return d * static_cast<float>(0.01745329251994329576923690768489); }
float degrees(float r) { return r * static_cast<float>(57.295779513082320876798154814105); }
} // namespace

// src/camera.cpp:11-19
PreviewCamera::PreviewCamera(vec3 position, vec3 lookAt, vec3 up) {
    const vec3 direction = normalize(position - lookAt);
    Position = position;
    WorldUp = up;
    Yaw = (float)::atan2((double)direction.x, (double)direction.z);
    Pitch = (float)(::asin((double)direction.y) + 1.57079632679);
    updateCameraVectors();
}

// src/camera.cpp:31-45
void PreviewCamera::ProcessKeyboard(CameraMovement direction, float deltaTime) {
    const float velocity = MovementSpeed * deltaTime;
    if (direction == FORWARD) Position = Position + Front * velocity;
    if (direction == BACKWARD) Position = Position - Front * velocity;
    if (direction == LEFT) Position = Position - Right * velocity;
    if (direction == RIGHT) Position = Position + Right * velocity;
    if (direction == UPWARD) Position = Position - Up * velocity;
    if (direction == DOWNWARD) Position = Position + Up * velocity;
}

// src/camera.cpp:47-63
void PreviewCamera::ProcessMouseMovement(float xoffset, float yoffset, bool constrainPitch) {
    xoffset *= MouseSensitivity;
    yoffset *= MouseSensitivity;
    Yaw += xoffset;
    Pitch += yoffset;
    if (constrainPitch) {
        if (Pitch > 89.0f) Pitch = 89.0f;
        if (Pitch < -89.0f) Pitch = -89.0f;
    }
    updateCameraVectors();
}

// src/camera.cpp:65-72
void PreviewCamera::ProcessMouseScroll(float yoffset) {
    if (Zoom >= 1.0f && Zoom <= 90.0f) Zoom -= yoffset;
    if (Zoom <= 1.0f) Zoom = 1.0f;
    if (Zoom >= 90.0f) Zoom = 90.0f;
}

// src/camera.cpp:74-85
void PreviewCamera::updateCameraVectors() {
    vec3 front;
    front.x = (float)(::cos((double)radians(Yaw)) * ::cos((double)radians(Pitch)));
    front.y = (float)::sin((double)radians(Pitch));
    front.z = (float)(::sin((double)radians(Yaw)) * ::cos((double)radians(Pitch)));
    Front = normalize(front);
    Right = normalize(cross(Front, WorldUp));
    Up = normalize(cross(Right, Front));
}

float preview_zoom(float yview) { return degrees(2.f * atanf(0.5f * yview)); }

// src/openglPreview.cpp:12-15, 39
PreviewSession::PreviewSession(Scene &s, RayTracer &r) : camera(s.VP, s.LA, s.UP), scene(s), renderer(r) {
    camera.Zoom = preview_zoom(scene.yview);
}

// src/openglPreview.cpp:139-146, 247-251
void PreviewSession::pressRender() {
    showRender = true;
    renderer.rayTrace(camera.Position, camera.Front + camera.Position, camera.Up,
                      (float)(2 * ::tan(camera.Zoom * M_PI / 360.)));
    renders++;
    updateScreen();
}

// src/openglPreview.cpp:156-173
void PreviewSession::exposureUp() {
    scene.exposure += 0.2;
    std::cout << "Scene exposure is now " << scene.exposure << std::endl;
    updateScreen();
}
void PreviewSession::exposureDown() {
    scene.exposure -= 0.2;
    std::cout << "Scene exposure is now " << scene.exposure << std::endl;
    updateScreen();
}

// src/openglPreview.cpp:178-197: the movement keys move at the speed the previous frame
// left, and only then does the frame set the speed from the shift key for the next one
void PreviewSession::move(CameraMovement d, float deltaTime, bool fast) {
    if (showRender) return;
    camera.ProcessKeyboard(d, deltaTime);
    camera.MovementSpeed = fast ? 30.f : 2.5f;
}
// a frame with no movement key (src/openglPreview.cpp:193-196 alone)
void PreviewSession::shiftState(bool fast) {
    if (showRender) return;
    camera.MovementSpeed = fast ? 30.f : 2.5f;
}
void PreviewSession::look(float xoffset, float yoffset) {
    if (!showRender) camera.ProcessMouseMovement(xoffset, yoffset);
}
void PreviewSession::scroll(float yoffset) {
    if (!showRender) camera.ProcessMouseScroll(yoffset);
}

// src/openglPreview.cpp:253-257 (the texture upload is the caller's)
const uint8_t *PreviewSession::updateScreen() {
    renderer.normalizeImage();
    return renderer.getData();
}

} // namespace chiaro
