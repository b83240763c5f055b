// Scene O of output_shader.frag:12-48 as a scene plugin:
//     rm_load_scene(ctx, "raymarching_amd/scenes/output_shader.hip")
// renders what the compiled-in "output_shader.frag" renders (a mirror Menger
// sponge, spun by u_time, smoothly merged with a blue sphere and cube and a
// checker floor), through the generic plugin path.  Written in the GLSL
// subset that rm_sdf_lib.h accepts.
const Material kMirror = Material(vec3(0.1), vec3(0.09), 64.0, 0.25, 0.0, vec3(0.0), 1.0, vec3(0.0));
const Material kBlue = Material(vec3(0.02, 0.02, 0.2), vec3(0.02, 0.02, 0.04), 32.0, 0.0, 0.0,
                                vec3(2.0, 2.0, 0.75) * 0.2, 1.52, vec3(0.0, 0.0, 100.0));

// black/white tiles whose edges are smoothed over a width that grows with
// the distance from the origin
Material checker(vec3 pos)
{
    float blur = max(10.0, pow(length(pos), 1.3));
    vec2 t = smoothstep(-0.005, 0.005, sin(pos.xz * PI) / blur);
    float tile = min(max(t.x, t.y), max(1.0 - t.x, 1.0 - t.y));
    return Material(mix(vec3(0.3), vec3(0.025), tile), vec3(0.03), 128.0, 0.0, 0.0, vec3(0.0), 1.0, vec3(0.0));
}

SdResult sceneSDF(vec3 p)
{
    vec3 q = transformR(p - vec3(0.0, 3.0, 0.0), vec3(180.0, u_time * 2.0, 0.0));
    SdResult sponge = SdResult(mengersponge(q).x, kMirror);
    SdResult ball = SdResult(sphere(vec4(3.0, 2.0, 3.0, 1.0), p), kBlue);
    SdResult box = SdResult(cube(vec4(-5.0, 4.0, 5.0, 1.0), p), kBlue);
    SdResult ground = SdResult(plane(p), checker(p));
    SdResult shapes = sminCubic(sminCubic(ball, box, 0.5), ground, 0.5);
    return sminCubic(sponge, shapes, 0.33);
}
