// The alternative scene the reference keeps commented out in its sceneSDF
// (output_shader.frag:41): a green mandelbulb, scaled by 1.5 and spun by
// u_time, in place of the Menger sponge, with the same sphere, cube and floor.
const Material kGreen = Material(vec3(0.02, 0.2, 0.02), vec3(0.02, 0.04, 0.02), 32.0, 0.0, 0.0, vec3(0.0), 1.0,
                                 vec3(0.0));
const Material kBlue = Material(vec3(0.02, 0.02, 0.2), vec3(0.02, 0.02, 0.04), 32.0, 0.0, 0.0,
                                vec3(2.0, 2.0, 0.75) * 0.2, 1.52, vec3(0.0, 0.0, 100.0));

Material checker(vec3 pos)
{
    float blur = max(10.0, pow(length(pos), 1.3));
    vec2 t = smoothstep(-0.005, 0.005, sin(pos.xz * PI) / blur);
    float tile = min(max(t.x, t.y), max(1.0 - t.x, 1.0 - t.y));
    return Material(mix(vec3(0.3), vec3(0.025), tile), vec3(0.03), 128.0, 0.0, 0.0, vec3(0.0), 1.0, vec3(0.0));
}

SdResult sceneSDF(vec3 p)
{
    vec4 orbit = vec4(1.0);
    vec3 q = transformRS1(p - vec3(0.0, 2.0, 0.0), vec3(180.0, u_time * 2.0, 0.0), 1.5);
    SdResult bulb = SdResult(mandelbulb(q, orbit) * 1.5, kGreen);
    SdResult ball = SdResult(sphere(vec4(3.0, 2.0, 3.0, 1.0), p), kBlue);
    SdResult box = SdResult(cube(vec4(-5.0, 4.0, 5.0, 1.0), p), kBlue);
    SdResult ground = SdResult(plane(p), checker(p));
    return sminCubic(bulb, sminCubic(sminCubic(ball, box, 0.5), ground, 0.5), 0.33);
}
